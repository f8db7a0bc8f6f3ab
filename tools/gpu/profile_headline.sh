#!/bin/bash
# rocprofv3 kernel trace + stats of the headline ResNet-50 b1024 step: serialised (wgrad on the main
# stream, overlap_wgrad=0: per-kernel times add up to the step) and the default schedule ("def": per-block side
# forks at this size); then per-kernel top list + timeline gaps.
set -o pipefail
O=${1:-gpurun_out/prof_headline}
mkdir -p $O
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for ov in 0 def; do
  ev="DBX_ENGINE=overlap_wgrad=$ov"; [ $ov = def ] && ev="DBX_ENGINE="
  (cd /tmp && env $ev timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/rp_ov$ov -o run --output-format csv -- python3 $R/bench.py --steps 6 --warmup 3 > $R/$O/rp_ov$ov.log 2>&1) || { echo "rocprof ov=$ov failed"; tail -5 $O/rp_ov$ov.log; exit 1; }
  grep -o '"value": [0-9.]*' $O/rp_ov$ov.log
  f=$(find $O/rp_ov$ov -name "*kernel_stats.csv" | head -1)
  t=$(find $O/rp_ov$ov -name "*kernel_trace.csv" | head -1)
  python3 tools/prof_top.py "$f" 9 60 > $O/top_ov$ov.txt 2>&1 || true
  python3 tools/trace_gaps.py "$t" --last 4 --top 20 > $O/gaps_ov$ov.txt 2>&1 || true
  head -45 $O/top_ov$ov.txt; head -12 $O/gaps_ov$ov.txt
done
