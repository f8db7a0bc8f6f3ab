#!/bin/bash
# Multi-rank one-graph step (world-1 RCCL) with and without the deferred side launch, loopback collectives on/off.
set -o pipefail
O=${1:-gpurun_out/side_defer_mr}
mkdir -p $O
W1="RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29733 DBX_FORCE_PG=1 DBX_SEGMENTED_GRAPHS=1"
for r in 1 2; do
  for p in headline resnet50_tiny_imagenet; do
    for st in "1 2" "0 2" "1 0" "0 0"; do
      set -- $st
      a="--steps 30 --warmup 10 --preset $p"; [ $p = headline ] && a="--steps 15 --warmup 5"
      f=$O/${p}_defer$1_lb$2_r$r.log
      env $W1 DBX_SIDE_DEFER=$1 DBX_COMM_LOOPBACK=$2 timeout -k 10 300 python3 bench.py --gpus 1 $a > $f 2>&1 || { tail -20 $f; exit 1; }
      echo "$p multirank defer=$1 loopback=$2 r$r: $(grep -o '"value": [0-9.]*' $f)"
    done
  done
done
