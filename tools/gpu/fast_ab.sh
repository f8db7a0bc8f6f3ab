#!/bin/bash
# Eight-wave conv kernel A/B on the compute-bound ResNet-50 b1024 shapes (tools/bench_fast.py).
set -o pipefail
O=${1:-gpurun_out/fast_ab}
mkdir -p $O
timeout -k 10 600 python -u tools/bench_fast.py --batch ${BATCH:-1024} --rounds 5 --iters 10 > $O/bench_fast.jsonl 2> $O/bench_fast.err
rc=$?
cat $O/bench_fast.jsonl | cut -c1-400
[ $rc = 0 ] || { tail -20 $O/bench_fast.err; exit $rc; }
