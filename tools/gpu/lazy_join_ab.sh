#!/bin/bash
# no intermediate side-stream joins (DBX_LAZY_JOIN=1): bit-identity + loopback post order, then A/B
set -o pipefail
O=${1:-gpurun_out/lazy_join}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_program_gpu.py tests/test_comm_gpu.py \
  -k "side_stream_bit_identical or loopback" > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || exit 1
W1="RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29733 DBX_FORCE_PG=1 DBX_SEGMENTED_GRAPHS=1"
for r in 1 2; do
  bash tools/gpu/sweep_env.sh $O/r$r "resnet50_tiny_imagenet resnet18_cifar10 headline" base DBX_LAZY_JOIN=1 DBX_LAZY_JOIN=1+DBX_SIDE_DEFER=1 || exit 1
  for p in resnet50_tiny_imagenet; do
    for l in 0 1; do
      f=$O/r$r/${p}_mr_lb_lazy$l.log
      env $W1 DBX_LAZY_JOIN=$l DBX_COMM_LOOPBACK=2 timeout -k 10 300 python3 bench.py --gpus 1 --preset $p --steps 30 --warmup 10 > $f 2>&1 || { tail -20 $f; exit 1; }
      echo "$p multirank loopback lazy=$l r$r: $(grep -o '"value": [0-9.]*' $f)"
    done
  done
done
