#!/bin/bash
# Kernel stats of eager steps without wgrad overlap (clean per-kernel times): rocprofv3 --stats
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/test_kernels.log 2>&1 || { echo "tests FAILED"; tail -30 gpurun_out/test_kernels.log; exit 1; }
tail -1 gpurun_out/test_kernels.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_eager -o run --output-format csv -- python3 $R/tools/op_breakdown.py --steps 3 --top 80 > $R/gpurun_out/op_breakdown_prof.txt 2>&1 || { echo "prof FAILED"; tail -20 $R/gpurun_out/op_breakdown_prof.txt; exit 1; }
cd $R && timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/bench.log 2>&1 || { echo "bench FAILED"; tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-200
