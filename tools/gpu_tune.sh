#!/bin/bash
# Tile tuning + numerics + A/B bench on one GPU.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu > gpurun_out/test_kernels.log 2>&1 || { echo "kernel tests FAILED"; tail -30 gpurun_out/test_kernels.log; exit 1; }
tail -1 gpurun_out/test_kernels.log
timeout -k 10 600 python tools/tune_conv.py --batch 1024 --report gpurun_out/tune_b1024.md > gpurun_out/tune.log 2>&1 || { echo "tune FAILED"; tail -30 gpurun_out/tune.log; exit 1; }
cp dbx_distributed_pytorch_examples_amd/ops/tune_table.json gpurun_out/tune_table.json
for m in none fwd all none fwd,dgrad0,dgrad2 all; do
DBX_TUNE_MODES=$m timeout -k 10 300 python bench.py --steps 20 --warmup 5 --batch 1024 > gpurun_out/ab_$m.log 2>&1 || { echo "bench $m FAILED"; tail -20 gpurun_out/ab_$m.log; exit 1; }
echo "$m: $(tail -1 gpurun_out/ab_$m.log | cut -c90-130)"
done
