#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu > gpurun_out/test_kernels.log 2>&1 || { tail -30 gpurun_out/test_kernels.log; exit 1; }
tail -1 gpurun_out/test_kernels.log
for d in 1 2; do DBX_WGRAD_DEPTH=$d timeout -k 10 300 python tools/tune_conv.py --modes wgrad --out gpurun_out/wg_table.json --report gpurun_out/tw_$d.md > gpurun_out/tw.log 2>&1 || exit 1; done
timeout -k 10 600 python tools/tune_conv.py --modes fwd,dgrad0,dgrad1,dgrad2 --out gpurun_out/tune_new.json --report gpurun_out/tune_pipe3.md > gpurun_out/tune.log 2>&1 || exit 1
cp gpurun_out/tune_new.json dbx_distributed_pytorch_examples_amd/ops/tune_table.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --batch 1024 > gpurun_out/bench_b1024.log 2>&1 || exit 1
tail -1 gpurun_out/bench_b1024.log | cut -c1-150
