#!/bin/bash
# Rehearse the multi-rank native path on ONE GPU over real RCCL: world-1 "nccl" process group with
# DBX_SEGMENTED_GRAPHS=1 forces per-segment graph capture + side-stream bucket all-reduces (the
# world > 1 code path) while the ProcessGroupNCCL watchdog runs. Checks graph == eager bit for bit,
# then times the headline bench segmented vs single-graph.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export DBX_FORCE_PG=1
L="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1"
DBX_SEGMENTED_GRAPHS=1 DBX_SEG_GROUPS=3,3 timeout -k 10 300 $L --master-port 29611 tools/dist_gpu_check.py > gpurun_out/rccl_check.log 2>&1 || { echo "rccl check FAILED"; tail -30 gpurun_out/rccl_check.log; exit 1; }
grep dist_gpu_check gpurun_out/rccl_check.log
DBX_SEGMENTED_GRAPHS=1 timeout -k 10 300 $L --master-port 29614 tools/dist_gpu_check.py > gpurun_out/rccl_check6.log 2>&1 || { echo "rccl check (6 segments) FAILED"; tail -30 gpurun_out/rccl_check6.log; exit 1; }
grep dist_gpu_check gpurun_out/rccl_check6.log
DBX_SEGMENTED_GRAPHS=1 timeout -k 10 300 $L --master-port 29615 bench.py --gpus 1 --steps 30 --warmup 10 > gpurun_out/rccl_bench_seg6.log 2>&1 || { echo "seg6 bench FAILED"; tail -30 gpurun_out/rccl_bench_seg6.log; exit 1; }
echo "6 segments+RCCL: $(tail -1 gpurun_out/rccl_bench_seg6.log | cut -c90-170)"
DBX_SEGMENTED_GRAPHS=1 DBX_SEG_GROUPS=3,3 timeout -k 10 300 $L --master-port 29612 bench.py --gpus 1 --steps 30 --warmup 10 > gpurun_out/rccl_bench_seg.log 2>&1 || { echo "seg bench FAILED"; tail -30 gpurun_out/rccl_bench_seg.log; exit 1; }
echo "2 segments+RCCL: $(tail -1 gpurun_out/rccl_bench_seg.log | cut -c90-170)"
timeout -k 10 300 $L --master-port 29613 bench.py --gpus 1 --steps 30 --warmup 10 > gpurun_out/rccl_bench_one.log 2>&1 || { echo "bench FAILED"; tail -30 gpurun_out/rccl_bench_one.log; exit 1; }
echo "single graph:   $(tail -1 gpurun_out/rccl_bench_one.log | cut -c90-170)"
