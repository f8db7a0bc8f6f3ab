#!/bin/bash
# Round 4: headline A/B of tune-table candidates (interleaved rounds): the repo table | + the re-tuned
# tail / fold / prologue entries (128x256 tail tiles, 4-slot rings) | + the 256x256 weight-gradient
# tile at one workgroup round; then the multi-rank benches.
set -o pipefail
O=${1:-gpurun_out/r4_s3}
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  for t in base t_tail t_tail_wg; do
    tt=""; [ $t != base ] && tt="DBX_TUNE_TABLE=tools/r4_tables/$t.json"
    env $tt timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/headline_${t}_$r.log 2>&1 \
      || { tail -20 $O/headline_${t}_$r.log; exit 1; }
    echo "headline $t r$r: $(grep -o '"value": [0-9.]*' $O/headline_${t}_$r.log)"
  done
done
bash tools/gpu/r4_comm_bench.sh $O/comm
