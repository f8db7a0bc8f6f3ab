#!/bin/bash
# LDS-DMA operand paths of the fwd / dgrad conv kernels: bit-exactness tests, tile x path tuning
# (written to gpurun_out, merged by hand), headline bench with the current table.
set -o pipefail
mkdir -p gpurun_out/r2s3
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_conv_dma_gpu.py > gpurun_out/r2s3/t_dma.log 2>&1 || { echo "dma tests FAILED"; tail -30 gpurun_out/r2s3/t_dma.log; exit 1; }
tail -2 gpurun_out/r2s3/t_dma.log
cp dbx_distributed_pytorch_examples_amd/ops/tune_table.json gpurun_out/r2s3/tune_dma.json
timeout -k 10 600 python tools/tune_conv.py --verbose --modes fwd,fwdt,dgrad0,dgrad1,dgrad2,dgrad1b,dgrad2b --out gpurun_out/r2s3/tune_dma.json --report gpurun_out/r2s3/tune_dma.md > gpurun_out/r2s3/tune_dma.log 2>&1 || { echo "tune FAILED"; tail -30 gpurun_out/r2s3/tune_dma.log; exit 1; }
echo tuned
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2s3/bench_before.log 2>&1 && tail -1 gpurun_out/r2s3/bench_before.log | cut -c1-130
DBX_TUNE_TABLE=gpurun_out/r2s3/tune_dma.json timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2s3/bench_dma.log 2>&1 && tail -1 gpurun_out/r2s3/bench_dma.log | cut -c1-130
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2s3/bench_before2.log 2>&1 && tail -1 gpurun_out/r2s3/bench_before2.log | cut -c1-130
DBX_TUNE_TABLE=gpurun_out/r2s3/tune_dma.json timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2s3/bench_dma2.log 2>&1 && tail -1 gpurun_out/r2s3/bench_dma2.log | cut -c1-130
