#!/bin/bash
# Which hardware queue the comm branch of the one-graph multi-rank step lands on (DEBUG_HIP_FORCE_GRAPH_QUEUES=2):
# world-1 RCCL one-graph step with DBX_COMM_LOOPBACK=2 (each bucket "all-reduce" is a scale kernel on the comm
# stream, visible in a kernel trace), traced by rocprofv3; tools/queue_report.py then lists per queue the kernel
# classes (comm scale / weight gradients / main chain).
set -o pipefail
O=${1:-gpurun_out/comm_queue}
mkdir -p $O
export TMPDIR=/tmp
RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29733 DBX_FORCE_PG=1 \
  DBX_SEGMENTED_GRAPHS=1 DBX_COMM_LOOPBACK=2 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
  -d $O/rp -o run -- python3 bench.py --gpus 1 --preset resnet50_tiny_imagenet --steps 6 --warmup 3 > $O/bench.log 2>&1 \
  || { tail -20 $O/bench.log; exit 1; }
python3 tools/queue_report.py $(find $O/rp -name "run_kernel_trace.csv" | head -1) > $O/queues.txt && cat $O/queues.txt
