#!/bin/bash
# LARS kernel + native LARS graph step, ZeRO-3, then the whole GPU suite, smoke and the headline bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_lars.py tests/test_zero3_cpu.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/test_new.log 2>&1 || { echo "new tests FAILED"; tail -40 gpurun_out/test_new.log; exit 1; }
tail -1 gpurun_out/test_new.log
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/test_gpu.log 2>&1 || { echo "gpu suite FAILED"; tail -40 gpurun_out/test_gpu.log; exit 1; }
tail -1 gpurun_out/test_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { echo "smoke FAILED"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/bench_default.log 2>&1 || { echo "bench FAILED"; tail -20 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log | cut -c1-200
