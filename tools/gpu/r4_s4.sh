#!/bin/bash
# Round 4: numerics of the row-tile kernel (tile code 7) and the world-1 framework-communicator test;
# a re-tune of the BN-prologue 1x1 entries (fwd / fwdt / dgrad1b / dgrad2b) with the row tile as a
# candidate into a COPY of the tune table; the headline with the repo table vs the copy (and the copy
# with every conv1 data gradient folded: DBX_FOLD_MAX_RATIO=8).
set -o pipefail
O=${1:-gpurun_out/r4_s4}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_rowtile_gpu.py tests/test_comm_gpu.py -x -q --timeout 120 \
  --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -4 $O/pytest.log; [ $rc = 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
T=dbx_distributed_pytorch_examples_amd/ops/tune_table.json
cp $T $O/tune_table.json
timeout -k 10 500 python -u tools/tune_conv.py --batch 1024 --rounds 3 --iters 3 --dma 1 --verbose \
  --modes fwd,fwdt,dgrad1b,dgrad2b --out $O/tune_table.json --report $O/tune_rowtile.md > $O/tune_rowtile.log 2>&1 \
  || { tail -20 $O/tune_rowtile.log; exit 1; }
grep -c "x7 |" $O/tune_rowtile.md || true
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/headline_base_$r.log 2>&1 || { tail -20 $O/headline_base_$r.log; exit 1; }
  echo "headline base r$r: $(grep -o '"value": [0-9.]*' $O/headline_base_$r.log)"
  DBX_TUNE_TABLE=$O/tune_table.json timeout -k 10 300 python bench.py --steps 20 --warmup 5 \
    > $O/headline_rt_$r.log 2>&1 || { tail -20 $O/headline_rt_$r.log; exit 1; }
  echo "headline rowtile r$r: $(grep -o '"value": [0-9.]*' $O/headline_rt_$r.log)"
  DBX_FOLD_MAX_RATIO=8 DBX_TUNE_TABLE=$O/tune_table.json timeout -k 10 300 python bench.py --steps 20 --warmup 5 \
    > $O/headline_rtf_$r.log 2>&1 || { tail -20 $O/headline_rtf_$r.log; exit 1; }
  echo "headline rowtile+fold-all r$r: $(grep -o '"value": [0-9.]*' $O/headline_rtf_$r.log)"
done
