#!/bin/bash
# Re-tune the headline's weight gradients (tile x operand path, then split depth) into a COPY of the
# tune table, then an interleaved headline A/B: the repo table vs the re-tuned copy.
set -o pipefail
O=${1:-gpurun_out/tune_wgrad_headline}
mkdir -p $O
T=dbx_distributed_pytorch_examples_amd/ops/tune_table.json
cp $T $O/tune_table.before.json
cp $T $O/tune_table.json
timeout -k 10 700 python tools/tune_conv.py --model resnet50 --batch 1024 --image 224 --modes wgrad --rounds 3 --iters 5 \
    --verbose --out $O/tune_table.json --report $O/report_tiles.md > $O/tune_tiles.log 2>&1 || { tail -20 $O/tune_tiles.log; exit 1; }
grep "^| " $O/tune_tiles.log
timeout -k 10 700 python tools/tune_conv.py --model resnet50 --batch 1024 --image 224 --modes wgrad --wgrad-rounds 0.5,1,2 \
    --rounds 3 --iters 5 --verbose --out $O/tune_table.json --report $O/report_rounds.md > $O/tune_rounds.log 2>&1 \
    || { tail -20 $O/tune_rounds.log; exit 1; }
grep "^| " $O/tune_rounds.log
for r in 1 2 3; do
  for tb in before new; do
    f=$O/tune_table.json; [ $tb = before ] && f=$O/tune_table.before.json
    DBX_ENGINE=tune_table=$f timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_${tb}_$r.log 2>&1 || { tail -20 $O/bench_${tb}_$r.log; exit 1; }
    echo "bench $tb r$r: $(grep -o '"value": [0-9.]*' $O/bench_${tb}_$r.log)"
  done
done
