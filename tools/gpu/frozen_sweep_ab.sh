#!/bin/bash
# frozen-backbone (inference-mode program) throughput with and without the sweep forward.
set -o pipefail
O=${1:-gpurun_out/frozen_sweep}; mkdir -p $O; export TMPDIR=/tmp
for r in 1 2; do
  for v in 1 0; do
    DBX_ENGINE=sweep_fwd=$v timeout -k 10 400 python tools/bench_frozen.py --impls native --configs r50_imagenet_b256,r50_tiny_mds,r50_imagenet_b32 --steps 30 --warmup 5 > $O/frozen_${v}_$r.log 2>&1 || { tail -20 $O/frozen_${v}_$r.log; exit 1; }
    grep '^{' $O/frozen_${v}_$r.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('sweep_fwd=$v r$r', d.get('config'), d.get('value') or d.get('images_per_s'))" | tee -a $O/ab.txt
  done
done
