#!/bin/bash
# Multi-rank path checks after the overlap change: 2 gloo ranks sharing the GPU (world 2 code
# path, bit-exact graph/eager/ZeRO-1) and the world-1 RCCL rehearsal.
set -o pipefail
mkdir -p gpurun_out
DBX_DIST_BACKEND=gloo timeout -k 10 400 python -m dbx_distributed_pytorch_examples_amd.launch --nproc-per-node 2 tools/dist_gpu_check.py > gpurun_out/dist_check.log 2>&1 || { echo "dist check FAILED"; tail -20 gpurun_out/dist_check.log; exit 1; }
grep "dist_gpu_check" gpurun_out/dist_check.log
bash tools/gpu_rccl_rehearsal.sh
