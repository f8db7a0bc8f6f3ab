#!/bin/bash
# kernels + program numerics, then native bench + rocprof
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu > gpurun_out/test_kernels.log 2>&1; echo "kernels rc=$?"; tail -3 gpurun_out/test_kernels.log
timeout -k 10 600 python -m pytest tests/test_program_gpu.py -x -q -m gpu > gpurun_out/test_program.log 2>&1; echo "program rc=$?"; tail -25 gpurun_out/test_program.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; echo "smoke rc=$?"; tail -3 gpurun_out/smoke.log
DBX_GRAPHS=0 timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_native_eager.log 2>&1; echo "bench eager rc=$?"; tail -2 gpurun_out/bench_native_eager.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_native.log 2>&1; echo "bench rc=$?"; tail -2 gpurun_out/bench_native.log
cd /tmp && DBX_GRAPHS=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_native -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof_native.log 2>&1; echo "prof rc=$?"
