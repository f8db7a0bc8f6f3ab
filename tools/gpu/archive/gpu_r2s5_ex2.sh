#!/bin/bash
# Re-run of the two examples that failed on the GPU in gpu_r2s5_allexamples.sh after their fixes.
set -o pipefail
O=gpurun_out/r2s5_examples_all
mkdir -p $O
E=examples
timeout -k 10 240 python -u $E/01_torch_distributor/01_basic_mnist.py --procs 1 --samples 512 --out /tmp/ex > $O/mnist.log 2>&1 || { echo "mnist FAILED"; tail -20 $O/mnist.log; exit 1; }
echo "mnist: $(tail -1 $O/mnist.log | cut -c1-150)"
timeout -k 10 240 python -u $E/04_accelerate/01_cifar_accelerate.py --native --samples 1024 --batch-size 128 --out /tmp/ex > $O/accelerate_native.log 2>&1 || { echo "accelerate native FAILED"; tail -20 $O/accelerate_native.log; exit 1; }
echo "accelerate_native: $(tail -1 $O/accelerate_native.log | cut -c1-150)"
