#!/bin/bash
# split-depth tuning of the ResNet-50 b256 224x224 weight gradients (the ZeRO-1 preset's shapes), then
# an interleaved ZeRO-1 preset A/B: new table vs the committed one
set -o pipefail
O=${1:-gpurun_out/tune_wr256}
mkdir -p $O
T=dbx_distributed_pytorch_examples_amd/ops/tune_table.json
cp $T $O/tune_table.before.json
cp $T $O/tune_table.json
timeout -k 10 500 python tools/tune_conv.py --model resnet50 --batch 256 --image 224 --modes wgrad --wgrad-rounds 0,0.5,1,2,4 \
    --rounds 3 --iters 5 --out $O/tune_table.json --report $O/report.md > $O/tune.log 2>&1 || { tail -20 $O/tune.log; exit 1; }
grep "^| " $O/tune.log | tail -n +1
for r in 1 2; do
  for tb in before new; do
    f=$O/tune_table.json; [ $tb = before ] && f=$O/tune_table.before.json
    DBX_ENGINE=tune_table=$f timeout -k 10 300 python bench.py --preset resnet50_imagenet_zero1 --steps 20 --warmup 5 > $O/bench_${tb}_$r.log 2>&1 || { tail -20 $O/bench_${tb}_$r.log; exit 1; }
    echo "zero1 $tb r$r: $(grep -o '"value": [0-9.]*' $O/bench_${tb}_$r.log)"
  done
done
