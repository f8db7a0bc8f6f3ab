#!/bin/bash
# world-1 RCCL rehearsal of the multi-rank (segmented-graph) step: headline / TinyImageNet benches of
# the segmented step with the side stream off (the world > 1 default), per block (3), per gradient (1).
set -o pipefail
O=${1:-gpurun_out/seg_overlap}
mkdir -p $O
export TMPDIR=/tmp DBX_FORCE_PG=1 DBX_SEGMENTED_GRAPHS=1
L="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1"
port=29630
for r in 1 2; do
  for p in headline resnet50_tiny_imagenet; do
    for m in off 3 1; do
      port=$((port + 1))
      ev=""; [ $m != off ] && ev="DBX_OVERLAP_WGRAD=$m"
      args="--steps 15 --warmup 5"; [ $p != headline ] && args="--steps 30 --warmup 10 --preset $p"
      env $ev timeout -k 10 300 $L --master-port $port bench.py --gpus 1 $args > $O/${p}_${m}_$r.log 2>&1 || { tail -20 $O/${p}_${m}_$r.log; exit 1; }
      echo "$p segmented overlap=$m r$r: $(grep -o '"value": [0-9.]*' $O/${p}_${m}_$r.log)"
    done
  done
done
