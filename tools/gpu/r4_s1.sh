#!/bin/bash
# Round 4, first measurement call: numerics of the new kernel paths (256x256 wgrad tile, 32-channel
# stage rings in the eight-wave and four-wave kernels, half-split TAIL prologue), native MNIST
# semantics, the world-1 RCCL rehearsal; the wgrad microbenchmark; a re-tune of the plain fwd / dgrad
# operand paths and of the eight-wave entries with the deep ring into a COPY of the tune table; the
# headline with the current table vs the re-tuned one.
set -o pipefail
O=${1:-gpurun_out/r4_s1}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_conv_fast_gpu.py tests/test_conv_dma_gpu.py \
  tests/test_mnist_native_gpu.py tests/test_multirank_gpu.py tests/test_comm_gpu.py -x -q --timeout 300 \
  --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -4 $O/pytest.log; [ $rc = 0 ] || { grep -E "FAILED|Error" $O/pytest.log | head; exit $rc; }
timeout -k 10 400 python -u tools/bench_wgrad_big.py --batch 1024 --rounds 3 > $O/bench_wgrad_big.txt 2>&1
rc=$?; cut -c1-330 $O/bench_wgrad_big.txt; [ $rc = 0 ] || exit $rc
T=dbx_distributed_pytorch_examples_amd/ops/tune_table.json
cp $T $O/tune_table.json
timeout -k 10 400 python -u tools/tune_conv.py --batch 1024 --rounds 3 --iters 3 --modes dgrad0,dgrad1,dgrad2,fwd,fwdt,dgrad1b,dgrad2b \
  --out $O/tune_table.json --report $O/tune_plain.md > $O/tune_plain.log 2>&1 || { tail -20 $O/tune_plain.log; exit 1; }
DBX_FAST_STAGE=32 timeout -k 10 300 python -u tools/tune_conv.py --batch 1024 --rounds 3 --iters 3 --fast 0.03 \
  --modes fwd0,dgrad1,dgrad2 --out $O/tune_table.json --report $O/tune_fast32.md > $O/tune_fast32.log 2>&1 \
  || { tail -20 $O/tune_fast32.log; exit 1; }
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/headline_base_$r.log 2>&1 || { tail -20 $O/headline_base_$r.log; exit 1; }
  echo "headline base r$r: $(grep -o '"value": [0-9.]*' $O/headline_base_$r.log)"
  DBX_FAST_STAGE=32 DBX_TUNE_TABLE=$O/tune_table.json timeout -k 10 300 python bench.py --steps 20 --warmup 5 \
    > $O/headline_new_$r.log 2>&1 || { tail -20 $O/headline_new_$r.log; exit 1; }
  echo "headline retuned+stage32 r$r: $(grep -o '"value": [0-9.]*' $O/headline_new_$r.log)"
done
