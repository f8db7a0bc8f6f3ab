#!/bin/bash
# split-depth tuning of every wgrad shape of the three bench configs, then bench A/B with the new table
set -o pipefail
O=${1:-gpurun_out/tune_wr}
mkdir -p $O
cp dbx_distributed_pytorch_examples_amd/ops/tune_table.json $O/tune_table.before.json
cp dbx_distributed_pytorch_examples_amd/ops/tune_table.json $O/tune_table.json
for cfg in "resnet18 256 32" "resnet50 512 64" "resnet50 1024 224"; do
  set -- $cfg
  timeout -k 10 400 python tools/tune_conv.py --model $1 --batch $2 --image $3 --modes wgrad --wgrad-rounds 0,0.5,1,2,4 \
      --rounds 3 --iters 5 --verbose --out $O/tune_table.json --report $O/report_$1_$2_$3.md > $O/tune_$1_$2_$3.log 2>&1 \
      || { tail -20 $O/tune_$1_$2_$3.log; exit 1; }
  grep "^| " $O/tune_$1_$2_$3.log | tail -n +1
done
cp $O/tune_table.json dbx_distributed_pytorch_examples_amd/ops/tune_table.json
for p in resnet18_cifar10 resnet50_tiny_imagenet headline; do
  args="--steps 30 --warmup 10 --preset $p"; [ $p = headline ] && args="--steps 15 --warmup 5"
  timeout -k 10 300 python bench.py $args > $O/bench_$p.log 2>&1 || { tail -20 $O/bench_$p.log; exit 1; }
  echo "$p tuned: $(grep -o '"value": [0-9.]*' $O/bench_$p.log)"
done
