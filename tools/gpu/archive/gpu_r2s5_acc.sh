#!/bin/bash
# Round-2 session-5: top-1 parity at 224 on a stable schedule (lr 0.02, two warmup epochs, 8 epochs),
# native engine (default fused kernel paths) vs the eager torch reference-equivalent, two task difficulties.
set -o pipefail
O=gpurun_out/r2s5acc
mkdir -p $O
for nz in 96 128; do
  A="--size 224 --train 12800 --val 2048 --epochs 8 --lr 0.02 --warmup-epochs 2 --noise $nz"
  timeout -k 10 500 python -u tools/accuracy_parity.py $A --json-out $O/acc224_lr0.02_noise$nz.json > $O/log_noise$nz.txt 2>&1 || { echo "noise $nz FAILED"; tail -5 $O/log_noise$nz.txt; exit 1; }
  echo "noise $nz:"; grep -E '"epoch": (4|8)' $O/log_noise$nz.txt | cut -c1-240
done
