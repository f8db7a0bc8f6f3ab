#!/bin/bash
# Round 4: 256 x 256 weight-gradient tile -- numerics vs fp32, then the per-shape microbenchmark.
set -o pipefail
O=${1:-gpurun_out/r4_wgrad}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 200 --timeout-method thread \
  -k "wgrad" > $O/pytest_wgrad.log 2>&1
rc=$?; tail -5 $O/pytest_wgrad.log; [ $rc = 0 ] || { grep -E "FAILED|Error" $O/pytest_wgrad.log | head; exit $rc; }
timeout -k 10 600 python -u tools/bench_wgrad_big.py --batch 1024 > $O/bench_wgrad_big.txt 2>&1
rc=$?; cat $O/bench_wgrad_big.txt | cut -c1-400; exit $rc
