#!/bin/bash
# Concurrent output phases of the strided dgrads (DBX_DGRAD_PHASE_STREAMS=1): program GPU tests with it on,
# then alternating benches on / off on the same box.
set -o pipefail
O=gpurun_out/r2s5_phase
mkdir -p $O
DBX_DGRAD_PHASE_STREAMS=1 timeout -k 10 400 python -u -m pytest tests/test_program_gpu.py tests/test_kernels_gpu.py -x -q -k "program or dgrad or frozen or native_module" --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { echo "tests FAILED"; tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
for r in 1 2 3; do
  for v in 0 1; do
    DBX_DGRAD_PHASE_STREAMS=$v timeout -k 10 300 python bench.py --steps 30 --warmup 10 > $O/bench_${v}_$r.log 2>&1 || { echo "bench FAILED"; tail -20 $O/bench_${v}_$r.log; exit 1; }
    echo "phase_streams=$v run $r: $(tail -1 $O/bench_${v}_$r.log | cut -c90-125)"
  done
done
