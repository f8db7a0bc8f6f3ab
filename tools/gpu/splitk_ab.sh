#!/bin/bash
# split-K of the few-tile convs: GPU tests (split-K numerics, the kernel / program suites that now run it),
# then interleaved bench A/B of splitk_wgs / splitk_min_kb on the small presets and the headline.
set -o pipefail
O=${1:-gpurun_out/splitk}; R=${2:-2}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_splitk_gpu.py \
  tests/test_kernels_gpu.py tests/test_program_gpu.py -m gpu > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for r in $(seq 1 $R); do
  bash tools/gpu/sweep_env.sh $O/r$r "resnet50_tiny_imagenet resnet18_cifar10" DBX_ENGINE=splitk_wgs=0 \
    DBX_ENGINE=splitk_wgs=512 DBX_ENGINE=splitk_wgs=1024 DBX_ENGINE=splitk_wgs=2048 \
    DBX_ENGINE=splitk_wgs=1024,splitk_min_kb=2 || exit 1
done
bash tools/gpu/sweep_env.sh $O/h "headline" base DBX_ENGINE=splitk_wgs=0 || exit 1
