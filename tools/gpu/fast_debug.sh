#!/bin/bash
set -o pipefail
O=${1:-gpurun_out/fast_debug}
mkdir -p $O
timeout -k 10 300 python -u tools/debug_fast_stats.py > $O/stats.log 2>&1; rc=$?; cat $O/stats.log | tail -30; exit $rc
