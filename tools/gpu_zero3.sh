#!/bin/bash
# ZeRO-3 GPU tests, then the whole GPU suite and the smoke step.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_zero3_cpu.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/test_zero3.log 2>&1 || { echo "zero3 FAILED"; tail -40 gpurun_out/test_zero3.log; exit 1; }
tail -1 gpurun_out/test_zero3.log
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/test_gpu.log 2>&1 || { echo "gpu suite FAILED"; tail -40 gpurun_out/test_gpu.log; exit 1; }
tail -1 gpurun_out/test_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { echo "smoke FAILED"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
