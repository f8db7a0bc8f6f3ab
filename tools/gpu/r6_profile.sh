#!/bin/bash
# Round-6 headline profile after the N-sweep forward: eager per-op table + op classes, rocprofv3 kernel
# stats / timeline of the graph-replayed default step.  usage: r6_profile.sh OUT
set -o pipefail
O=${1:-gpurun_out/r6_prof}; mkdir -p $O; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
BATCH=1024 timeout -k 10 300 python -u tools/op_breakdown.py --steps 2 --top 80 > $O/op_breakdown.txt 2>&1 || { tail -20 $O/op_breakdown.txt; exit 1; }
python3 tools/op_classes.py $O/op_breakdown.txt > $O/op_classes.txt 2>&1 || true
head -12 $O/op_classes.txt
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/rp_def -o run --output-format csv -- python3 $R/bench.py --steps 6 --warmup 3 > $R/$O/rp_def.log 2>&1) || { echo "rocprof failed"; tail -5 $O/rp_def.log; exit 1; }
f=$(find $O/rp_def -name "*kernel_stats.csv" | head -1)
t=$(find $O/rp_def -name "*kernel_trace.csv" | head -1)
python3 tools/prof_top.py "$f" 9 60 > $O/top_def.txt 2>&1 || true
python3 tools/step_timeline.py "$t" --steps 2 --tail 0 > $O/timeline_def.txt 2>&1 || true
python3 tools/trace_gaps.py "$t" --last 4 --top 20 > $O/gaps_def.txt 2>&1 || true
head -30 $O/top_def.txt
rm -rf $O/rp_def/*/*.csv.gz 2>/dev/null; true
