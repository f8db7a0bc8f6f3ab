#!/bin/bash
# Tile tables for the preset shapes (the committed table only holds the b1024 ImageNet shapes): tune the
# ResNet-50 b256 224 (ZeRO-1 preset), ResNet-50 b512 64x64 (TinyImageNet preset) and ResNet-18 b256 32x32
# (CIFAR preset) shapes, merge ONLY keys absent from the committed table, then A/B old vs merged.
set -o pipefail
O=gpurun_out/r2s5_tunep
mkdir -p $O
export TMPDIR=/tmp
T=dbx_distributed_pytorch_examples_amd/ops/tune_table.json
for cfg in "resnet50 256 224 r50b256" "resnet50 512 64 r50tiny" "resnet18 256 32 r18cifar"; do
  set -- $cfg
  echo '{}' > $O/t_$4.json
  timeout -k 10 600 python -u tools/tune_conv.py --model $1 --batch $2 --image $3 --out $O/t_$4.json --report $O/t_$4.md > $O/t_$4.log 2>&1 || { echo "tune $4 FAILED"; tail -20 $O/t_$4.log; exit 1; }
done
python3 - <<'PY'
import json
O="gpurun_out/r2s5_tunep"
base=json.load(open("dbx_distributed_pytorch_examples_amd/ops/tune_table.json"))
m=dict(base); added=0; clash=0
for n in ("r50b256","r50tiny","r18cifar"):
    for k,v in json.load(open(f"{O}/t_{n}.json")).items():
        if k in m:
            clash+=1
        else:
            m[k]=v; added+=1
json.dump(m,open(f"{O}/merged.json","w"),indent=1,sort_keys=True)
print(f"merged: {len(base)} committed + {added} new entries ({clash} keys already tuned at b1024 kept)")
PY
for r in 1 2; do
  for t in old new; do
    if [ $t = new ]; then export DBX_TUNE_TABLE=$O/merged.json; else unset DBX_TUNE_TABLE; fi
    for p in resnet50_imagenet_zero1 resnet50_tiny_imagenet resnet18_cifar10; do
      timeout -k 10 300 python bench.py --preset $p --steps 20 --warmup 5 > $O/b_${p}_${t}_$r.log 2>&1 || { echo "bench FAILED"; tail -20 $O/b_${p}_${t}_$r.log; exit 1; }
      echo "$t run $r $p: $(tail -1 $O/b_${p}_${t}_$r.log | cut -c90-125)"
    done
  done
done
