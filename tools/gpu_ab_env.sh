#!/bin/bash
# A/B the headline bench over an environment switch, interleaved rounds: gpu_ab_env.sh VAR "v1 v2" [rounds]
set -o pipefail
mkdir -p gpurun_out
VAR=$1; VALS=$2; R=${3:-2}
for r in $(seq 1 $R); do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/ab_${VAR}_$v.log 2>&1 || { echo "bench $v FAILED"; tail -20 gpurun_out/ab_${VAR}_$v.log; exit 1; }
    echo "round $r $VAR=$v: $(tail -1 gpurun_out/ab_${VAR}_$v.log | cut -c90-140)"
  done
done
