#!/bin/bash
# Round 4: the ping-pong eight-wave kernel (DBX_FAST_PP=1): bit-exactness against the four-wave
# kernel, per-shape A/B against the barrier-per-stage eight-wave kernel, headline A/B.
set -o pipefail
O=${1:-gpurun_out/r4_s5}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_conv_fast_gpu.py -x -q --timeout 120 --timeout-method thread \
  > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc = 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
timeout -k 10 400 python -u tools/bench_fast.py --pp --rounds 3 --iters 5 > $O/bench_fast_pp.txt 2>&1
rc=$?; cut -c1-600 $O/bench_fast_pp.txt; [ $rc = 0 ] || exit $rc
for r in 1 2; do
  for v in 0 1; do
    DBX_FAST_PP=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/headline_pp${v}_$r.log 2>&1 \
      || { tail -20 $O/headline_pp${v}_$r.log; exit 1; }
    echo "headline DBX_FAST_PP=$v r$r: $(grep -o '"value": [0-9.]*' $O/headline_pp${v}_$r.log)"
  done
done
