#!/bin/bash
# eight-wave kernel candidates for the plain-operand stride-1 fwd0 / dgrad1 / dgrad2 convs of the
# headline config (tools/tune_conv.py --fast), then an interleaved bench A/B: new table vs the old one
set -o pipefail
O=${1:-gpurun_out/tune_fast}
B=${2:-1024}                       # batch of the ResNet-50 224x224 shapes tuned
BENCH=${3:-"--steps 15 --warmup 5"}  # bench.py arguments of the A/B (default: the headline)
mkdir -p $O
T=dbx_distributed_pytorch_examples_amd/ops/tune_table.json
cp $T $O/tune_table.before.json
cp $T $O/tune_table.json
timeout -k 10 600 python tools/tune_conv.py --model resnet50 --batch $B --image 224 --modes fwd0,dgrad1,dgrad2 --fast 0.04 \
    --rounds 3 --iters 5 --verbose --out $O/tune_table.json --report $O/report.md > $O/tune.log 2>&1 || { tail -20 $O/tune.log; exit 1; }
grep "^| \|  \(fwd0\|dgrad\)" $O/tune.log
for r in 1 2; do
  for tb in before new; do
    f=$O/tune_table.json; [ $tb = before ] && f=$O/tune_table.before.json
    DBX_ENGINE=tune_table=$f timeout -k 10 300 python bench.py $BENCH > $O/bench_${tb}_$r.log 2>&1 || { tail -20 $O/bench_${tb}_$r.log; exit 1; }
    echo "bench $tb r$r: $(grep -o '"value": [0-9.]*' $O/bench_${tb}_$r.log)"
  done
done
