#!/bin/bash
# headline knob re-check after the round-6 changes (interleaved rounds; "default" repeated).
set -o pipefail
O=${1:-gpurun_out/head_knobs}; R=${2:-2}; mkdir -p $O; export TMPDIR=/tmp
V=("" "side_cu_reserve=96" "side_cu_reserve=160" "block_tail_main=1" "block_tail_main=3" "ds_fwd_side=0" "fold_min_elems=16777216" "fold_max_ratio=2" "fin_in=1" "coeff_in=1" "nshard=16" "wgrad_rounds=1.5" "wgrad_rounds=3" "lazy_join=0" "side_defer=0" "fuse_dw_min_hw=56")
for r in $(seq 1 $R); do
  for v in "${V[@]}"; do
    n=${v//[,=.]/_}; n=${n:-default}
    DBX_ENGINE=$v timeout -k 10 300 python bench.py --steps 15 --warmup 5 > $O/b_${n}_$r.log 2>&1 || { echo "FAIL $v"; tail -3 $O/b_${n}_$r.log; continue; }
    echo "headline ${v:-default} r$r: $(grep -o '"value": [0-9.]*' $O/b_${n}_$r.log)" | tee -a $O/ab.txt
  done
done
