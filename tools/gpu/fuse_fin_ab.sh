#!/bin/bash
# producer-side in-launch BN finalize (fuse_fin) re-measured on the three presets
set -o pipefail
O=${1:-gpurun_out/fuse_fin}; R=${2:-2}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_bn_fin_gpu.py tests/test_program_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc = 0 ] || { grep -E "FAILED|Error" $O/pytest.log | head; exit $rc; }
for r in $(seq 1 $R); do
  for p in resnet50_tiny_imagenet resnet18_cifar10 headline; do
    for v in "" "fuse_fin=1"; do
      n=${v//[,=]/_}; n=${n:-default}
      args="--steps 20 --warmup 5"; [ $p != headline ] && args="$args --preset $p"
      DBX_ENGINE=$v timeout -k 10 300 python bench.py $args > $O/b_${p}_${n}_$r.log 2>&1 || { echo "FAIL $p $v"; tail -3 $O/b_${p}_${n}_$r.log; continue; }
      echo "$p ${v:-default} r$r: $(grep -o '"value": [0-9.]*' $O/b_${p}_${n}_$r.log)" | tee -a $O/ab.txt
    done
  done
done
