#!/bin/bash
# Fwd / dgrad tile + operand-path tuning for the small-map presets (TinyImageNet ResNet-50 b512 @64,
# CIFAR ResNet-18 b256 @32: no fwd / dgrad entries before, the heuristic tile picked), then the
# eight-wave pass, then an interleaved A/B of the new table against the in-tree one.
set -o pipefail
O=${1:-gpurun_out/tune_small}
mkdir -p $O
T=$O/table.json
cp dbx_distributed_pytorch_examples_amd/ops/tune_table.json $T
M="fwd,fwdt,dgrad0,dgrad1,dgrad2,dgrad1b,dgrad2b"
timeout -k 10 400 python tools/tune_conv.py --model resnet50 --batch 512 --image 64 --modes $M --out $T --report $O/tiny.md > $O/tiny.log 2>&1 || { tail $O/tiny.log; exit 1; }
timeout -k 10 300 python tools/tune_conv.py --model resnet50 --batch 512 --image 64 --fast 0.04 --out $T --report $O/tiny_fast.md > $O/tiny_fast.log 2>&1 || { tail $O/tiny_fast.log; exit 1; }
timeout -k 10 300 python tools/tune_conv.py --model resnet18 --batch 256 --image 32 --modes $M --out $T --report $O/cifar.md > $O/cifar.log 2>&1 || { tail $O/cifar.log; exit 1; }
timeout -k 10 300 python tools/tune_conv.py --model resnet18 --batch 256 --image 32 --fast 0.04 --out $T --report $O/cifar_fast.md > $O/cifar_fast.log 2>&1 || { tail $O/cifar_fast.log; exit 1; }
for r in 1 2; do
  for p in resnet50_tiny_imagenet resnet18_cifar10; do
    for v in new old; do
      if [ $v = new ]; then tt=$T; else tt=dbx_distributed_pytorch_examples_amd/ops/tune_table.json; fi
      DBX_ENGINE=tune_table=$tt timeout -k 10 300 python bench.py --preset $p --steps 30 --warmup 10 > $O/${p}_${v}_r$r.log 2>&1 || { tail -20 $O/${p}_${v}_r$r.log; exit 1; }
      echo "$p $v r$r: $(grep -o '"value": [0-9.]*' $O/${p}_${v}_r$r.log)"
    done
  done
done
