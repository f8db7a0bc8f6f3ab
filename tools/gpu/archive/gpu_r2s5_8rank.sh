#!/bin/bash
# 8-rank (and a 2-rank bit-exactness check) rehearsal of the driver's multi-GPU bench command on ONE GPU: every rank on
# cuda:0, gloo as the process-group backend (RCCL refuses duplicate devices), small per-rank batch so
# 8 ranks fit one card. Exercises: rendezvous, initial broadcast, segmented graphs + comm-stream
# bucket all-reduces at world 8, ZeRO-1 reduce/all-gather at world 8, barrier + max-elapsed, rank-0 line.
set -o pipefail
O=gpurun_out/r2s5_8rank
mkdir -p $O
export DBX_DIST_BACKEND=gloo
L="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
timeout -k 10 400 $L --nproc-per-node 8 --master-port 29731 bench.py --gpus 8 --batch 32 --steps 4 --warmup 3 > $O/dp8.log 2>&1 || { echo "dp8 FAILED"; tail -30 $O/dp8.log; exit 1; }
echo "dp8: $(grep '"metric"' $O/dp8.log | cut -c80-200)"
timeout -k 10 400 $L --nproc-per-node 8 --master-port 29732 bench.py --gpus 8 --preset resnet50_imagenet_zero1 --batch 32 --steps 4 --warmup 3 > $O/zero1_dp8.log 2>&1 || { echo "zero1 dp8 FAILED"; tail -30 $O/zero1_dp8.log; exit 1; }
echo "zero1 dp8: $(grep '"metric"' $O/zero1_dp8.log | cut -c80-200)"
timeout -k 10 300 $L --nproc-per-node 2 --master-port 29733 tools/dist_gpu_check.py > $O/check2.log 2>&1 || { echo "dist check 2 FAILED"; tail -30 $O/check2.log; exit 1; }
grep dist_gpu_check $O/check2.log
