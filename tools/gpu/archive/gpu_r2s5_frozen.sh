#!/bin/bash
# Frozen-backbone head training (the reference's TD / DS ResNet workloads): native (graph-replayed
# backbone), native eager (DBX_FROZEN_GRAPHS=0) and the reference-equivalent torch stack.
set -o pipefail
O=gpurun_out/r2s5_frozen
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_program_gpu.py -x -q -k frozen --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { echo "tests FAILED"; tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 500 python -u tools/bench_frozen.py --steps 30 --warmup 5 > $O/frozen.txt 2>&1 || { echo "bench_frozen FAILED"; tail -20 $O/frozen.txt; exit 1; }
DBX_FROZEN_GRAPHS=0 timeout -k 10 300 python -u tools/bench_frozen.py --steps 30 --warmup 5 --impls native > $O/frozen_eager.txt 2>&1 || { echo "bench_frozen eager FAILED"; tail -20 $O/frozen_eager.txt; exit 1; }
grep images_per_s $O/frozen.txt | cut -c1-150
echo "native eager:"; grep images_per_s $O/frozen_eager.txt | cut -c1-150
