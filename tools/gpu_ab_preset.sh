#!/bin/bash
# A/B a preset bench over an environment switch: gpu_ab_preset.sh PRESET VAR "v1 v2" [rounds]
set -o pipefail
mkdir -p gpurun_out
P=$1; VAR=$2; VALS=$3; R=${4:-2}
for r in $(seq 1 $R); do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 300 python bench.py --preset $P --steps 20 --warmup 5 > gpurun_out/abp_${VAR}_$v.log 2>&1 || { echo "bench $v FAILED"; tail -20 gpurun_out/abp_${VAR}_$v.log; exit 1; }
    echo "round $r $P $VAR=$v: $(tail -1 gpurun_out/abp_${VAR}_$v.log | cut -c90-140)"
  done
done
