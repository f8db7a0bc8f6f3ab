#!/bin/bash
# Deferred forward BN statistics (one flush per persistent workgroup): kernel tests, stats probe, A/B.
set -o pipefail
O=gpurun_out/r2s4_defer
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_conv_dma_gpu.py tests/test_conv_patch3_gpu.py tests/test_program_gpu.py -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { echo "tests FAILED"; tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
for d in 1 0; do
  DBX_STATS_DEFER=$d timeout -k 10 300 python tools/probe_stats.py > $O/probe_defer$d.txt 2>&1 || { echo "probe FAILED"; tail -5 $O/probe_defer$d.txt; exit 1; }
  echo "defer=$d"; grep -v amdgpu.ids $O/probe_defer$d.txt | head -4
done
for r in 1 2; do
  for d in 1 0; do
    DBX_STATS_DEFER=$d timeout -k 10 300 python bench.py --steps 30 --warmup 10 > $O/bench_d${d}_r$r.log 2>&1 || { echo "bench FAILED"; tail -20 $O/bench_d${d}_r$r.log; exit 1; }
    echo "defer=$d run $r: $(tail -1 $O/bench_d${d}_r$r.log | cut -c80-130)"
  done
done
