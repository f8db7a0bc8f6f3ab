#!/bin/bash
# The multi-rank step (world-1 RCCL group, segmented path forced) vs the single graph on the three
# presets: plain | segmented c10d (late posts + side stream) | one-graph framework comm | segmented
# c10d without the side stream (round-3 layout).
set -o pipefail
O=${1:-gpurun_out/r4_comm}
mkdir -p $O
export TMPDIR=/tmp
L="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1"
port=29640
for p in resnet18_cifar10 resnet50_tiny_imagenet headline; do
  args="--steps 30 --warmup 10 --preset $p"; [ $p = headline ] && args="--steps 15 --warmup 5"
  timeout -k 10 300 python bench.py $args > $O/${p}_plain.log 2>&1 || { tail -20 $O/${p}_plain.log; exit 1; }
  echo "$p plain: $(grep -o '"value": [0-9.]*' $O/${p}_plain.log)"
  for c in torch native torch_noside; do
    port=$((port + 1))
    side=1; cm=$c; [ $c = torch_noside ] && { side=0; cm=torch; }
    DBX_FORCE_PG=1 DBX_SEGMENTED_GRAPHS=1 DBX_COMM=$cm DBX_SEG_SIDE=$side timeout -k 10 300 $L --master-port $port \
      bench.py --gpus 1 $args > $O/${p}_seg_$c.log 2>&1 || { tail -20 $O/${p}_seg_$c.log; exit 1; }
    echo "$p segmented comm=$c: $(grep -o '"value": [0-9.]*' $O/${p}_seg_$c.log)"
  done
done
