#!/bin/bash
# Re-tune conv tiles at batch 1024 (all modes), then bench with the new table.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u tools/tune_conv.py --batch 1024 --report gpurun_out/tune_b1024.md > gpurun_out/tune.log 2>&1 || { echo "tune FAILED"; tail -30 gpurun_out/tune.log; exit 1; }
cp dbx_distributed_pytorch_examples_amd/ops/tune_table.json gpurun_out/tune_table.json
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/bench.log 2>&1 || { echo "bench FAILED"; tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-200
