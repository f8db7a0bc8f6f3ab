#!/bin/bash
# Step-level tile tuning of one preset (tools/tune_step.py), then an interleaved A/B of the tuned table
# against the tree's:  tune_step.sh OUT PRESET BUDGET_S ROUNDS
set -o pipefail
O=${1:-gpurun_out/tune_step}; P=${2:-resnet50_tiny_imagenet}; B=${3:-420}; R=${4:-3}
mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 $((B + 240)) python -u tools/tune_step.py --preset $P --budget-s $B --out $O/tune_$P.json \
  > $O/tune_$P.log 2>&1 || { tail -30 $O/tune_$P.log; exit 1; }
tail -1 $O/tune_$P.log | cut -c1-400
args="--steps 30 --warmup 10"; [ $P = headline ] && args="--steps 15 --warmup 5" || args="$args --preset $P"
for r in $(seq 1 $R); do
  for v in tree tuned; do
    e="DBX_ENGINE="; [ $v = tuned ] && e="DBX_ENGINE=tune_table=$O/tune_$P.json"
    env $e timeout -k 10 300 python bench.py $args > $O/${P}_${v}_r$r.log 2>&1 || { tail -20 $O/${P}_${v}_r$r.log; exit 1; }
    echo "$P $v r$r: $(grep -o '"value": [0-9.]*' $O/${P}_${v}_r$r.log)"
  done
done
