#!/bin/bash
# Collectives on the weight-gradient side stream (DBX_COMM_SIDE=1) vs their own stream (=0) in the one-graph
# multi-rank step: the loopback post-order tests, the queue report, then world-1 RCCL bench lines with a real
# collective in the graph (DBX_COMM_LOOPBACK=2) and without.
set -o pipefail
O=${1:-gpurun_out/comm_side}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_comm_gpu.py tests/test_multirank_gpu.py > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || exit 1
W1="RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29733 DBX_FORCE_PG=1 DBX_SEGMENTED_GRAPHS=1"
env $W1 DBX_COMM_LOOPBACK=2 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
  -d $O/rp -o run -- python3 bench.py --gpus 1 --preset resnet50_tiny_imagenet --steps 6 --warmup 3 > $O/trace.log 2>&1 \
  || { tail -20 $O/trace.log; exit 1; }
python3 tools/queue_report.py $(find $O/rp -name "run_kernel_trace.csv" | head -1) | tee $O/queues.txt
for r in 1 2; do
  for p in resnet50_tiny_imagenet resnet18_cifar10 headline; do
    for st in "1 2" "0 2" "1 0"; do
      set -- $st
      a="--steps 30 --warmup 10 --preset $p"; [ $p = headline ] && a="--steps 15 --warmup 5"
      f=$O/${p}_side$1_lb$2_r$r.log
      env $W1 DBX_COMM_SIDE=$1 DBX_COMM_LOOPBACK=$2 timeout -k 10 300 python3 bench.py --gpus 1 $a > $f 2>&1 || { tail -20 $f; exit 1; }
      echo "$p comm_side=$1 loopback=$2 r$r: $(grep -o '"value": [0-9.]*' $f)"
    done
  done
done
