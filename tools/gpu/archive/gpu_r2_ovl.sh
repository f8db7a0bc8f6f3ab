#!/bin/bash
# wgrad side-stream overlap on/off, plain single graph vs segmented multi-rank path (world-1 RCCL
# rehearsal), two interleaved rounds.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
port=29690
for r in 1 2; do
for ov in 1 0; do
  export DBX_OVERLAP_WGRAD=$ov
  unset RANK LOCAL_RANK WORLD_SIZE LOCAL_WORLD_SIZE MASTER_ADDR MASTER_PORT DBX_FORCE_PG DBX_SEGMENTED_GRAPHS
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/ovl_plain.log 2>&1 || { echo "plain FAILED"; tail -20 gpurun_out/ovl_plain.log; exit 1; }
  echo "overlap=$ov plain:     $(tail -1 gpurun_out/ovl_plain.log | cut -c80-150)"
  port=$((port+1))
  export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=$port DBX_FORCE_PG=1 DBX_SEGMENTED_GRAPHS=1
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/ovl_seg.log 2>&1 || { echo "seg FAILED"; tail -20 gpurun_out/ovl_seg.log; exit 1; }
  echo "overlap=$ov segmented: $(tail -1 gpurun_out/ovl_seg.log | cut -c80-150)"
done
done
