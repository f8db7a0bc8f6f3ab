#!/bin/bash
# Probe: two ranks on ONE GPU over RCCL (both on cuda:0). If RCCL accepts a duplicate device, the
# multi-rank native path (segmented graphs + side-stream RCCL all-reduces) runs for real.
set -o pipefail
mkdir -p gpurun_out
L="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
NCCL_DEBUG=WARN timeout -k 10 180 $L --master-port 29641 tools/dist_gpu_check.py > gpurun_out/rccl2_check.log 2>&1; rc=$?
echo "rccl 2-rank check rc=$rc"; grep -E "dist_gpu_check|Error|error|Duplicate|WARN" gpurun_out/rccl2_check.log | head -20
