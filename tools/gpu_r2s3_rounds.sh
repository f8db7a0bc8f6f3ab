#!/bin/bash
# wgrad split-K workgroup rounds A/B (DBX_WGRAD_ROUNDS): fewer rounds = smaller fp32 partial slabs
set -o pipefail
mkdir -p gpurun_out/r2s3
for r in 1 2; do
  for v in 2 1 1.5; do
    DBX_WGRAD_ROUNDS=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2s3/rounds_$v.log 2>&1 || { echo "bench $v FAILED"; tail -20 gpurun_out/r2s3/rounds_$v.log; exit 1; }
    echo "wgrad_rounds=$v: $(tail -1 gpurun_out/r2s3/rounds_$v.log | cut -c80-140)"
  done
done
DBX_WGRAD_ROUNDS=1 timeout -k 10 300 python bench.py --preset resnet50_tiny_imagenet --steps 20 --warmup 5 > gpurun_out/r2s3/rounds_t1.log 2>&1 && echo "tiny rounds=1: $(tail -1 gpurun_out/r2s3/rounds_t1.log | cut -c80-140)"
timeout -k 10 300 python bench.py --preset resnet50_tiny_imagenet --steps 20 --warmup 5 > gpurun_out/r2s3/rounds_t2.log 2>&1 && echo "tiny rounds=2: $(tail -1 gpurun_out/r2s3/rounds_t2.log | cut -c80-140)"
