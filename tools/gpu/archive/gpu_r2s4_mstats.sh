#!/bin/bash
# Forward BN statistics on the matrix cores (igemm epilogue): kernel tests, stats probe, bench.
set -o pipefail
O=gpurun_out/r2s4_mstats
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_conv_dma_gpu.py tests/test_conv_patch3_gpu.py tests/test_program_gpu.py -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { echo "tests FAILED"; tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 300 python tools/probe_stats.py > $O/probe.txt 2>&1 || { echo "probe FAILED"; tail -5 $O/probe.txt; exit 1; }
grep -v amdgpu.ids $O/probe.txt
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 10 > $O/bench_r$r.log 2>&1 || { echo "bench FAILED"; tail -20 $O/bench_r$r.log; exit 1; }
  echo "run $r: $(tail -1 $O/bench_r$r.log | cut -c1-140)"
done
