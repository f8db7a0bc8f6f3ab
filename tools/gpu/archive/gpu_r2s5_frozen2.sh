#!/bin/bash
# Frozen-backbone whole-step graph (world 1, Adam): GPU tests, then native (whole-step graph), native with the
# backbone-only graph (DBX_FROZEN_FULL_GRAPH=0) on the reference's configs.
set -o pipefail
O=gpurun_out/r2s5_frozen2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_program_gpu.py -x -q -k frozen --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { echo "tests FAILED"; tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 400 python -u tools/bench_frozen.py --steps 30 --warmup 5 --impls native > $O/frozen_full.txt 2>&1 || { echo "bench_frozen FAILED"; tail -20 $O/frozen_full.txt; exit 1; }
DBX_FROZEN_FULL_GRAPH=0 timeout -k 10 400 python -u tools/bench_frozen.py --steps 30 --warmup 5 --impls native > $O/frozen_bb.txt 2>&1 || { echo "bench_frozen bb FAILED"; tail -20 $O/frozen_bb.txt; exit 1; }
echo "whole-step graph:"; grep images_per_s $O/frozen_full.txt | cut -c1-150
echo "backbone graph:"; grep images_per_s $O/frozen_bb.txt | cut -c1-150
