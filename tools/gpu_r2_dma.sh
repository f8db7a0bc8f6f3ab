#!/bin/bash
# LDS-DMA wgrad: numerics, per-shape tile x operand-path tuning at b1024, end-to-end A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "wgrad" > gpurun_out/t_wgrad.log 2>&1 || { echo "wgrad tests FAILED"; tail -30 gpurun_out/t_wgrad.log; exit 1; }
tail -1 gpurun_out/t_wgrad.log
cp dbx_distributed_pytorch_examples_amd/ops/tune_table.json gpurun_out/tune_table.json
timeout -k 10 400 python tools/tune_conv.py --modes wgrad --batch 1024 --out gpurun_out/tune_table.json --report gpurun_out/tune_wgrad_dma.md > gpurun_out/tune_wgrad.log 2>&1 || { echo "tune FAILED"; tail -20 gpurun_out/tune_wgrad.log; exit 1; }
cat gpurun_out/tune_wgrad_dma.md
for r in 1 2; do
  for v in 0 auto; do
    if [ $v = auto ]; then unset DBX_WGRAD_DMA; else export DBX_WGRAD_DMA=$v; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_dma_$v.log 2>&1 || { echo "bench $v FAILED"; tail -20 gpurun_out/bench_dma_$v.log; exit 1; }
    echo "dma=$v: $(tail -1 gpurun_out/bench_dma_$v.log | cut -c80-160)"
  done
done
unset DBX_WGRAD_DMA
DBX_TUNE_TABLE=gpurun_out/tune_table.json timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_dma_tuned.log 2>&1 && echo "tuned: $(tail -1 gpurun_out/bench_dma_tuned.log | cut -c80-160)"
