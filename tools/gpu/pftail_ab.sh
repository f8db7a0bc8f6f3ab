#!/bin/bash
# persistent forward tail kernels (DBX_PF_TAIL) A/B: tail tests, then interleaved presets.
# usage: pftail_ab.sh OUT ROUNDS   (base = production _C, nopft = -D DBX_PF_TAIL=0)
set -o pipefail
O=${1:-gpurun_out/pftail}; R=${2:-2}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_conv_dma_gpu.py tests/test_program_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc = 0 ] || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit $rc; }
for r in $(seq 1 $R); do
  for v in base nopft; do
    ev=""; [ $v != base ] && ev="DBX_EXT_VARIANT=$v"
    for p in headline resnet50_tiny_imagenet resnet50_imagenet_zero1; do
      args="--steps 15 --warmup 5"; [ $p != headline ] && args="$args --preset $p"
      env $ev timeout -k 10 300 python bench.py $args > $O/bench_${p}_${v}_$r.log 2>&1 || { tail -20 $O/bench_${p}_${v}_$r.log; exit 1; }
      echo "$p $v r$r: $(grep -o '"value": [0-9.]*' $O/bench_${p}_${v}_$r.log)" | tee -a $O/ab.txt
    done
  done
done
