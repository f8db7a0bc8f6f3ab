#!/bin/bash
# Round-3 GPU validation: full GPU test suite (incl. the multi-rank gloo-on-one-GPU checks), smoke,
# and the headline bench line. Usage: tools/gpu/check.sh OUTDIR
set -o pipefail
O=${1:-gpurun_out/check}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc = 0 ] || { grep -E "FAILED|Error|error" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '"metric"' $O/bench.log | cut -c1-260
timeout -k 10 300 python bench.py --preset resnet50_imagenet_zero1 --steps 20 --warmup 5 > $O/bench_zero1.log 2>&1 || { tail -20 $O/bench_zero1.log; exit 1; }
grep '"metric"' $O/bench_zero1.log | cut -c1-200
