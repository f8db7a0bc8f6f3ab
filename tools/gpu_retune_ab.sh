#!/bin/bash
# Re-tune conv tiles (modes in $1, default all) into a candidate table, then A/B old vs new table.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
MODES=${1:-fwd,dgrad0,dgrad1,dgrad2,wgrad}
cp dbx_distributed_pytorch_examples_amd/ops/tune_table.json gpurun_out/tune_old.json
cp dbx_distributed_pytorch_examples_amd/ops/tune_table.json gpurun_out/tune_new.json
timeout -k 10 900 python -u tools/tune_conv.py --batch 1024 --modes $MODES --out gpurun_out/tune_new.json --report gpurun_out/tune_b1024.md > gpurun_out/tune.log 2>&1 || { echo "tune FAILED"; tail -30 gpurun_out/tune.log; exit 1; }
for r in 1 2; do
  for t in old new; do
    DBX_TUNE_TABLE=gpurun_out/tune_$t.json timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/ab_$t.log 2>&1 || { echo "bench $t FAILED"; tail -20 gpurun_out/ab_$t.log; exit 1; }
    echo "round $r $t: $(tail -1 gpurun_out/ab_$t.log | cut -c90-140)"
  done
done
