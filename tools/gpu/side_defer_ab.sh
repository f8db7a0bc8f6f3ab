#!/bin/bash
# Deferred side-batch launch (DBX_SIDE_DEFER=1): bit-identity + loopback post-order tests, queue reports of the
# world-1 single-graph step and the one-graph multi-rank step with loopback collectives, then bench A/B.
set -o pipefail
O=${1:-gpurun_out/side_defer}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_program_gpu.py tests/test_comm_gpu.py \
  -k "side_stream_bit_identical or loopback" > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || exit 1
W1="RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29733 DBX_FORCE_PG=1 DBX_SEGMENTED_GRAPHS=1"
DBX_SIDE_DEFER=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/rp1 -o run -- python3 bench.py \
  --preset resnet50_tiny_imagenet --steps 6 --warmup 3 > $O/trace1.log 2>&1 || { tail -20 $O/trace1.log; exit 1; }
echo "== world 1, single graph, defer"; python3 tools/queue_report.py $(find $O/rp1 -name "run_kernel_trace.csv" | head -1) | tee $O/queues_single.txt
env $W1 DBX_SIDE_DEFER=1 DBX_COMM_LOOPBACK=2 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/rp2 -o run -- python3 bench.py \
  --gpus 1 --preset resnet50_tiny_imagenet --steps 6 --warmup 3 > $O/trace2.log 2>&1 || { tail -20 $O/trace2.log; exit 1; }
echo "== one-graph multi-rank, loopback, defer"; python3 tools/queue_report.py $(find $O/rp2 -name "run_kernel_trace.csv" | head -1) | tee $O/queues_multirank.txt
for r in 1 2; do
  bash tools/gpu/sweep_env.sh $O/r$r "resnet50_tiny_imagenet resnet18_cifar10 headline" base DBX_SIDE_DEFER=1 || exit 1
  for p in resnet50_tiny_imagenet resnet18_cifar10; do
    for d in 0 1; do
      f=$O/r$r/${p}_lb_defer$d.log
      env $W1 DBX_SIDE_DEFER=$d DBX_COMM_LOOPBACK=2 timeout -k 10 300 python3 bench.py --gpus 1 --preset $p --steps 30 --warmup 10 > $f 2>&1 || { tail -20 $f; exit 1; }
      echo "$p multirank loopback defer=$d r$r: $(grep -o '"value": [0-9.]*' $f)"
    done
  done
done
