#!/bin/bash
# Fused conv3 backward for the 28x28 stage: tests, kernel microbench per config variant, end-to-end A/B.
set -o pipefail
O=gpurun_out/r2s4_dwf5
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_dwfused_gpu.py -x -v --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { echo "dwfused tests FAILED"; tail -40 $O/test.log; exit 1; }
tail -2 $O/test.log
for v in "" n4 b32o3 b32n2o3; do
  DBX_EXT_VARIANT=$v timeout -k 10 200 python tools/bench_dwfused.py > $O/micro_$v.log 2>&1 || { echo "micro $v FAILED"; tail -20 $O/micro_$v.log; exit 1; }
  echo "variant '$v':"; cat $O/micro_$v.log | grep -v amdgpu.ids
done
for r in 1 2; do
  for f in 1 0; do
    DBX_FUSE_DW=$f timeout -k 10 300 python bench.py --steps 30 --warmup 10 > $O/bench_f${f}_r$r.log 2>&1 || { echo "bench FAILED"; tail -20 $O/bench_f${f}_r$r.log; exit 1; }
    echo "fuse=$f run $r: $(tail -1 $O/bench_f${f}_r$r.log | cut -c60-150)"
  done
done
