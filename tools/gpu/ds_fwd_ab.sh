#!/bin/bash
# downsample conv forward on the side stream beside conv2 / conv3 (DBX_DS_FWD_SIDE=1): bit-identity,
# one-step timeline, A/B on the headline and TinyImageNet
set -o pipefail
O=${1:-gpurun_out/ds_fwd}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_program_gpu.py -k "side_stream_bit_identical and dsf" > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || exit 1
DBX_DS_FWD_SIDE=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/rp -o run -- python3 bench.py --steps 6 --warmup 3 > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
python3 tools/step_timeline.py $(find $O/rp -name "*kernel_trace.csv" | head -1) --steps 1 --tail 0 --gap-us 300 --top-gaps 4 | head -12
for r in 1 2; do
  bash tools/gpu/sweep_env.sh $O/r$r "headline resnet50_tiny_imagenet" base DBX_DS_FWD_SIDE=1 || exit 1
done
