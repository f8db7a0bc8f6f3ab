#!/bin/bash
# One-graph multi-rank layouts at world 1 over a real RCCL group (a real collective kernel in the graph:
# comm_loopback=2) against the single-graph step: multirank_layout=block (per-block forks, per-segment
# posts) vs batch (round 5's batched layout with late posts). multirank_layout_ab.sh OUT "presets" ROUNDS
set -o pipefail
O=${1:-gpurun_out/mr_layout}; PRESETS=${2:-"headline resnet50_tiny_imagenet"}; R=${3:-2}
mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_comm_gpu.py \
  tests/test_multirank_gpu.py > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || exit $rc
port=29741
for r in $(seq 1 $R); do
  for p in $PRESETS; do
    a="--steps 15 --warmup 5"; [ $p != headline ] && a="--steps 30 --warmup 10 --preset $p"
    timeout -k 10 300 python bench.py $a > $O/${p}_single_r$r.log 2>&1 || { tail -20 $O/${p}_single_r$r.log; exit 1; }
    echo "$p single-graph r$r: $(grep -o '"value": [0-9.]*' $O/${p}_single_r$r.log)"
    for lay in block batch; do
      port=$((port + 1))
      DBX_FORCE_PG=1 DBX_ENGINE=segmented_graphs=1,comm_loopback=2,multirank_layout=$lay timeout -k 10 300 \
        python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $port \
        bench.py --gpus 1 $a > $O/${p}_${lay}_r$r.log 2>&1 || { tail -20 $O/${p}_${lay}_r$r.log; exit 1; }
      echo "$p one-graph $lay r$r: $(grep -o '"value": [0-9.]*' $O/${p}_${lay}_r$r.log)"
    done
  done
done
