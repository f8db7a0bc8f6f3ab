#!/bin/bash
# The one-graph multi-rank step's queue layout: queue report of the world-1 RCCL step with DBX_COMM_LOOPBACK=2 under
# DEBUG_HIP_FORCE_GRAPH_QUEUES=2 and =3, then bench lines of the same step (headline / TinyImageNet) per setting.
set -o pipefail
O=${1:-gpurun_out/comm_queue_ab}
mkdir -p $O
export TMPDIR=/tmp
W1="RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29733 DBX_FORCE_PG=1 DBX_SEGMENTED_GRAPHS=1"
for q in 2 3; do
  env $W1 DEBUG_HIP_FORCE_GRAPH_QUEUES=$q DBX_COMM_LOOPBACK=2 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
    -d $O/rp_q$q -o run -- python3 bench.py --gpus 1 --preset resnet50_tiny_imagenet --steps 6 --warmup 3 > $O/trace_q$q.log 2>&1 \
    || { tail -20 $O/trace_q$q.log; exit 1; }
  echo "== queues $q"; python3 tools/queue_report.py $(find $O/rp_q$q -name "run_kernel_trace.csv" | head -1) | tee $O/queues_q$q.txt
done
for r in 1 2; do
  for p in resnet50_tiny_imagenet headline; do
    for st in "2 0" "2 2" "3 0" "3 2"; do
      set -- $st
      a="--steps 30 --warmup 10 --preset $p"; [ $p = headline ] && a="--steps 15 --warmup 5"
      f=$O/${p}_q$1_lb$2_r$r.log
      env $W1 DEBUG_HIP_FORCE_GRAPH_QUEUES=$1 DBX_COMM_LOOPBACK=$2 timeout -k 10 300 python3 bench.py --gpus 1 $a > $f 2>&1 || { tail -20 $f; exit 1; }
      echo "$p queues=$1 loopback=$2 r$r: $(grep -o '"value": [0-9.]*' $f)"
    done
  done
done
