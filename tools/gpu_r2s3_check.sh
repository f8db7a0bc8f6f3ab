#!/bin/bash
# Round-2 session-3 revalidation on one GPU: GPU tests, smoke, headline bench, kernel stats.
set -o pipefail
mkdir -p gpurun_out/r2s3
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r2s3/test_gpu.log 2>&1 || { echo "GPU tests FAILED"; tail -40 gpurun_out/r2s3/test_gpu.log; exit 1; }
tail -1 gpurun_out/r2s3/test_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2s3/smoke.log 2>&1 || { echo "smoke FAILED"; tail -20 gpurun_out/r2s3/smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2s3/bench_default.log 2>&1 || { echo "bench FAILED"; tail -20 gpurun_out/r2s3/bench_default.log; exit 1; }
tail -1 gpurun_out/r2s3/bench_default.log
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r2s3/prof_b1024 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/r2s3/prof_b1024.log 2>&1; echo "prof rc=$?"
