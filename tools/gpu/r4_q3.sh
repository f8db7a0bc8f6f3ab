#!/bin/bash
# Graph-launch crash triage: the one-graph world-1 RCCL check under DEBUG_HIP_FORCE_GRAPH_QUEUES=$Q,
# then (if it passes) the small presets under the same setting.
set -o pipefail
O=${1:-gpurun_out/r4_q3}
Q=${2:-4}
mkdir -p $O
export DEBUG_HIP_FORCE_GRAPH_QUEUES=$Q
DBX_COMM=native DBX_FORCE_PG=1 DBX_SEGMENTED_GRAPHS=1 timeout -k 10 300 python -m dbx_distributed_pytorch_examples_amd.launch \
  --nproc-per-node 1 tools/dist_gpu_check.py > $O/check_q$Q.log 2>&1 || { tail -3 $O/check_q$Q.log; exit 1; }
tail -1 $O/check_q$Q.log
for p in resnet18_cifar10 resnet50_tiny_imagenet headline; do
  args="--steps 20 --warmup 5"; [ $p != headline ] && args="$args --preset $p"
  timeout -k 10 300 python bench.py $args > $O/${p}_q$Q.log 2>&1 || { tail -20 $O/${p}_q$Q.log; exit 1; }
  echo "$p q=$Q: $(grep -o '"value": [0-9.]*' $O/${p}_q$Q.log)"
done
