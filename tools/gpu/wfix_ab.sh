set -o pipefail
O=gpurun_out/r6_wfix; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_program_gpu.py -m gpu > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
bash tools/gpu/ab_variant_presets.sh $O old "headline resnet50_tiny_imagenet resnet18_cifar10" 2
