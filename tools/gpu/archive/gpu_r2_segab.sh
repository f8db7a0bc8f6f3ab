#!/bin/bash
# Multi-rank step layouts rehearsed over a world-1 RCCL process group on one GPU (DBX_FORCE_PG=1,
# DBX_SEGMENTED_GRAPHS=1 = the world > 1 code path): per-segment graphs (6), two groups (3,3),
# one backward graph + all-reduce after it (6), vs the plain single graph. Two rounds, interleaved.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 DBX_FORCE_PG=1
port=29650
for r in 1 2; do
  for g in "" "3,3" "6" "single"; do
    port=$((port+1)); export MASTER_PORT=$port
    if [ "$g" = single ]; then unset DBX_SEGMENTED_GRAPHS DBX_SEG_GROUPS; else export DBX_SEGMENTED_GRAPHS=1 DBX_SEG_GROUPS=$g; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/segab_$r.log 2>&1 || { echo "bench $g FAILED"; tail -20 gpurun_out/segab_$r.log; exit 1; }
    echo "groups=[${g:-per-segment}]: $(tail -1 gpurun_out/segab_$r.log | cut -c80-150)"
  done
done
