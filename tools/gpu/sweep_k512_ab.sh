#!/bin/bash
# 64-row-block sweep forwards (K 320-512): tests, probe, headline / ZeRO A/B against sweep_max_k=256
set -o pipefail
O=${1:-gpurun_out/sweep_k512}; R=${2:-2}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_sweep_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc = 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
timeout -k 10 200 python - > $O/probe.txt 2>&1 <<'PY'
import math, sys, torch
sys.path.insert(0, ".")
sys.argv = ["x"]
from tools.probe_sweep import fwd_case
for H, IC, OC, N in ((7, 512, 2048, 1024), (14, 512, 1024, 256), (7, 512, 2048, 256)):
    t0 = min(fwd_case(N, H, IC, OC, (128, 256, 1), 10) for _ in range(3))
    t1 = min(fwd_case(N, H, IC, OC, (128, 256, 8), 10) for _ in range(3))
    print(f"fwd {IC}->{OC} @{H} b{N}: igemm {t0*1e3:.1f} us  sweep {t1*1e3:.1f} us  {t0/t1:.2f}x", flush=True)
PY
grep fwd $O/probe.txt
for r in $(seq 1 $R); do
  for v in "" "sweep_max_k=256"; do
    for p in headline resnet50_imagenet_zero1; do
      n=${v//[,=]/_}; n=${n:-default}
      args="--steps 15 --warmup 5"; [ $p != headline ] && args="$args --preset $p"
      DBX_ENGINE=$v timeout -k 10 300 python bench.py $args > $O/b_${p}_${n}_$r.log 2>&1 || { echo "FAIL $p $v"; continue; }
      echo "$p ${v:-default} r$r: $(grep -o '"value": [0-9.]*' $O/b_${p}_${n}_$r.log)" | tee -a $O/ab.txt
    done
  done
done
