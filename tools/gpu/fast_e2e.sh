#!/bin/bash
# eight-wave kernel: its GPU tests, then the headline bench with / without it (interleaved runs)
set -o pipefail
O=${1:-gpurun_out/fast_e2e}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_conv_fast_gpu.py tests/test_mnist_native_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc = 0 ] || { grep -E "Error|assert" $O/pytest.log | head -20; exit $rc; }
for r in 1 2; do
  for f in 1 0; do
    DBX_FAST=$f timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_fast${f}_r$r.log 2>&1 || { tail -20 $O/bench_fast${f}_r$r.log; exit 1; }
    echo "fast=$f round $r: $(grep -o '"value": [0-9.]*' $O/bench_fast${f}_r$r.log)"
  done
done
