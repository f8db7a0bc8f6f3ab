#!/bin/bash
# rocprofv3 kernel stats of the small-shape presets (graph-replayed steps) + their bench lines.
set -o pipefail
O=${1:-gpurun_out/prof_presets}
mkdir -p $O
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for p in resnet18_cifar10 resnet50_tiny_imagenet; do
  timeout -k 10 300 python bench.py --preset $p --steps 30 --warmup 10 > $O/bench_$p.log 2>&1 || { tail -5 $O/bench_$p.log; exit 1; }
  echo "$p: $(grep -o '"value": [0-9.]*' $O/bench_$p.log) $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$p.log)"
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/rp_$p -o run --output-format csv -- python3 $R/bench.py --preset $p --steps 10 --warmup 3 > $R/$O/rp_$p.log 2>&1) || { echo "rocprof $p failed"; tail -5 $O/rp_$p.log; exit 1; }
  f=$(find $O/rp_$p -name "*kernel_stats.csv" | head -1)
  python3 tools/prof_top.py "$f" 13 > $O/top_$p.txt 2>&1 || true
  head -40 $O/top_$p.txt
done
