#!/bin/bash
# engine.native_module (native HIP program inside a user-written autograd loop): GPU test + throughput vs the
# stock torch module in the same loop (Accelerate / Ray / Composer notebook shapes).
set -o pipefail
O=gpurun_out/r2s5_nm
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_program_gpu.py -x -q -k native_module --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { echo "tests FAILED"; tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 500 python -u tools/bench_native_module.py --steps 20 --warmup 5 > $O/bench.txt 2>&1 && DBX_NATIVE_MODULE_GRAPHS=0 timeout -k 10 500 python -u tools/bench_native_module.py --steps 20 --warmup 5 --configs accelerate_r50_cifar,ray_r18_cifar > $O/bench_eager.txt 2>&1 || { echo "bench FAILED"; tail -20 $O/bench.txt; exit 1; }
grep images_per_s $O/bench.txt | cut -c1-140
echo "eager native module:"; grep images_per_s $O/bench_eager.txt | grep native | cut -c1-140
