#!/bin/bash
# Re-tune the conv tile x operand-path table at b1024 on the current kernels, then A/B the new table against
# the committed one (DBX_TUNE_TABLE) with alternating benches on the same box.
set -o pipefail
O=gpurun_out/r2s5_tune
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u tools/tune_conv.py --batch 1024 --out $O/tune_table.json --report $O/tune_b1024.md > $O/tune.log 2>&1 || { echo "tune FAILED"; tail -30 $O/tune.log; exit 1; }
echo "tuned: $(python3 -c "import json;print(len(json.load(open('$O/tune_table.json'))))") entries"
for r in 1 2 3; do
  for t in old new; do
    if [ $t = new ]; then export DBX_TUNE_TABLE=$O/tune_table.json; else unset DBX_TUNE_TABLE; fi
    timeout -k 10 300 python bench.py --steps 30 --warmup 10 > $O/bench_${t}_$r.log 2>&1 || { echo "bench FAILED"; tail -20 $O/bench_${t}_$r.log; exit 1; }
    echo "table=$t run $r: $(tail -1 $O/bench_${t}_$r.log | cut -c90-125)"
  done
done
