#!/bin/bash
# Round 4, first measurement call: numerics of the new kernel paths (256x256 wgrad tile, fast-kernel
# 32-channel stages, half-split TAIL prologue), native MNIST semantics, the world-1 RCCL rehearsal;
# then the wgrad microbenchmark, a headline A/B of the fast-kernel stage depth, the multi-rank
# (segmented / one-graph) step vs the single graph.
set -o pipefail
O=${1:-gpurun_out/r4_s1}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_conv_fast_gpu.py tests/test_mnist_native_gpu.py \
  tests/test_multirank_gpu.py tests/test_comm_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -4 $O/pytest.log; [ $rc = 0 ] || { grep -E "FAILED|Error" $O/pytest.log | head; exit $rc; }
timeout -k 10 600 python -u tools/bench_wgrad_big.py --batch 1024 --rounds 3 > $O/bench_wgrad_big.txt 2>&1
rc=$?; cut -c1-330 $O/bench_wgrad_big.txt; [ $rc = 0 ] || exit $rc
for r in 1 2; do
  for st in 64 32; do
    DBX_FAST_STAGE=$st timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/headline_st${st}_$r.log 2>&1 \
      || { tail -20 $O/headline_st${st}_$r.log; exit 1; }
    echo "headline fast-stage=$st r$r: $(grep -o '"value": [0-9.]*' $O/headline_st${st}_$r.log)"
  done
done
bash tools/gpu/r4_comm_bench.sh $O
