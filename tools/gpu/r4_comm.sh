#!/bin/bash
# Round 4: the world-1 RCCL rehearsal of every RCCL-only branch (c10d and framework communicator,
# DP and ZeRO-1), then the segmented multi-rank step vs the single-graph step on the three presets:
# plain (no process group) | segmented c10d (DBX_COMM=torch) | one-graph framework comm (DBX_COMM=native).
set -o pipefail
O=${1:-gpurun_out/r4_comm}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_multirank_gpu.py tests/test_comm_gpu.py -x -v --timeout 300 \
  --timeout-method thread -k "dist_check_rccl or comm" > $O/pytest_rccl.log 2>&1
rc=$?; tail -15 $O/pytest_rccl.log; [ $rc = 0 ] || exit $rc
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
