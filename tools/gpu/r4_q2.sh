#!/bin/bash
# Graph-launch crash triage: the one-graph world-1 RCCL check without / with the deferred reduce,
# and the CIFAR preset with the cumulative reduce-arena sizing.
set -o pipefail
O=${1:-gpurun_out/r4_q2}
mkdir -p $O
export DBX_COMM=native DBX_FORCE_PG=1 DBX_SEGMENTED_GRAPHS=1
DBX_DEFER_REDUCE=0 timeout -k 10 300 python -m dbx_distributed_pytorch_examples_amd.launch --nproc-per-node 1 \
  tools/dist_gpu_check.py > $O/check_nodefer.log 2>&1 || { tail -5 $O/check_nodefer.log; exit 1; }
tail -1 $O/check_nodefer.log
unset DBX_COMM DBX_FORCE_PG DBX_SEGMENTED_GRAPHS
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --preset resnet18_cifar10 > $O/cifar_$i.log 2>&1 || { tail -20 $O/cifar_$i.log; exit 1; }
  echo "cifar: $(grep -o '"value": [0-9.]*' $O/cifar_$i.log)"
done
DBX_COMM=native DBX_FORCE_PG=1 DBX_SEGMENTED_GRAPHS=1 timeout -k 10 300 python -m dbx_distributed_pytorch_examples_amd.launch \
  --nproc-per-node 1 tools/debug/run_bt.py tools/dist_gpu_check.py > $O/check_defer.log 2>&1 || { grep -A6 "segv_bt\]" $O/check_defer.log; tail -3 $O/check_defer.log; exit 1; }
tail -1 $O/check_defer.log
