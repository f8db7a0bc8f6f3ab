#!/bin/bash
# optimizer inside the backward (+ the small steps' BN-backward fold threshold): GPU bit-identity tests,
# then interleaved A/B of the settings
set -o pipefail
O=${1:-gpurun_out/r6_optbw}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_program_gpu.py -k "optimizer_in_backward or side_stream_bit_identical" > $O/pytest.txt 2>&1; rc=$?; tail -2 $O/pytest.txt; [ $rc = 0 ] || exit $rc
for r in 1 2; do
  bash tools/gpu/sweep_env.sh $O/r$r "resnet18_cifar10 resnet50_tiny_imagenet" DBX_ENGINE=overlap_optimizer=0 DBX_ENGINE=overlap_optimizer=2 DBX_ENGINE=overlap_optimizer=3 DBX_ENGINE=overlap_optimizer=4 DBX_ENGINE=overlap_optimizer=0,fold_min_elems=4194304 DBX_ENGINE=overlap_optimizer=0,fold_min_elems=0 || exit 1
  bash tools/gpu/sweep_env.sh $O/r$r "headline" DBX_ENGINE=overlap_optimizer=0 DBX_ENGINE=overlap_optimizer=3 || exit 1
done
