#!/bin/bash
# Accuracy parity at 224 (ResNet-50, 100 classes, b256) per kernel-path switch set.
set -o pipefail
O=gpurun_out/acc224
mkdir -p $O
A="--size 224 --train 12800 --val 2048 --epochs 4 --noise 160"
DBX_FUSE_DW=0 DBX_STEM_WGRAD=generic timeout -k 10 400 python -u tools/accuracy_parity.py $A --json-out $O/acc_nofuse.json > $O/log_nofuse.txt 2>&1 || { echo "nofuse FAILED"; tail -5 $O/log_nofuse.txt; exit 1; }
grep '"epoch": 4' $O/log_nofuse.txt | head -1 | cut -c1-200
DBX_FUSE_DW=0 DBX_STEM_WGRAD=generic DBX_PATCH3=0 DBX_STEM_PATCH=0 timeout -k 10 400 python -u tools/accuracy_parity.py $A --json-out $O/acc_nopatch.json > $O/log_nopatch.txt 2>&1 || { echo "nopatch FAILED"; tail -5 $O/log_nopatch.txt; exit 1; }
grep '"epoch": 4' $O/log_nopatch.txt | head -1 | cut -c1-200
