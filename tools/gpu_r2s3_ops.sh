#!/bin/bash
# Per-op breakdown (eager, hipEvent per wrapper) of the ResNet-50 b1024 native step.
set -o pipefail
mkdir -p gpurun_out/r2s3
timeout -k 10 300 python tools/op_breakdown.py --steps 3 --top 90 > gpurun_out/r2s3/op_breakdown.txt 2>&1 || { echo "op_breakdown FAILED"; tail -20 gpurun_out/r2s3/op_breakdown.txt; exit 1; }
head -30 gpurun_out/r2s3/op_breakdown.txt
