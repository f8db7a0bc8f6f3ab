#!/bin/bash
# Does the segmented multi-rank step lose its wgrad/dgrad overlap to hardware-queue sharing?
# HIP maps streams onto GPU_MAX_HW_QUEUES (default 4) hardware queues round-robin; the comm
# stream + RCCL's stream can push the wgrad side stream onto the main stream's queue.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
port=29670
for q in 4 8 16; do
  export GPU_MAX_HW_QUEUES=$q
  unset RANK LOCAL_RANK WORLD_SIZE LOCAL_WORLD_SIZE MASTER_ADDR MASTER_PORT DBX_FORCE_PG DBX_SEGMENTED_GRAPHS
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/hwq_plain_$q.log 2>&1 || { echo "plain $q FAILED"; tail -20 gpurun_out/hwq_plain_$q.log; exit 1; }
  echo "hwq=$q plain:     $(tail -1 gpurun_out/hwq_plain_$q.log | cut -c80-150)"
  port=$((port+1))
  export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=$port DBX_FORCE_PG=1 DBX_SEGMENTED_GRAPHS=1
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/hwq_seg_$q.log 2>&1 || { echo "seg $q FAILED"; tail -20 gpurun_out/hwq_seg_$q.log; exit 1; }
  echo "hwq=$q segmented: $(tail -1 gpurun_out/hwq_seg_$q.log | cut -c80-150)"
done
