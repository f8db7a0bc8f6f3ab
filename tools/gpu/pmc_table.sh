#!/bin/bash
# PMC table: per-kernel counters of one eager in-order b1024 step (four
# passes, tools/gpu/pmc_step.sh), the per-op roofline breakdown of the same configuration, and the
# kernel stats of the small presets.
set -o pipefail
O=${1:-gpurun_out/pmc_table}
mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu/pmc_step.sh 1024 $O/pmc || exit 1
BATCH=1024 timeout -k 10 300 python -u tools/op_breakdown.py --steps 2 --top 80 > $O/op_breakdown.txt 2>&1 \
  || { tail -20 $O/op_breakdown.txt; exit 1; }
head -30 $O/op_breakdown.txt
bash tools/gpu/profile_presets.sh $O/presets
