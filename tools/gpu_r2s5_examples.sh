#!/bin/bash
# The Accelerate notebook example on the GPU, stock module vs --native (engine.native_module), plus the
# frozen / native-module GPU tests.
set -o pipefail
O=gpurun_out/r2s5_examples
mkdir -p $O
timeout -k 10 300 python -u examples/04_accelerate/01_cifar_accelerate.py --samples 2048 --batch-size 128 --epochs 2 --out /tmp/acc_t > $O/accel_torch.log 2>&1 || { echo "accelerate torch FAILED"; tail -20 $O/accel_torch.log; exit 1; }
tail -2 $O/accel_torch.log
timeout -k 10 300 python -u examples/04_accelerate/01_cifar_accelerate.py --native --samples 2048 --batch-size 128 --epochs 2 --out /tmp/acc_n > $O/accel_native.log 2>&1 || { echo "accelerate native FAILED"; tail -20 $O/accel_native.log; exit 1; }
tail -2 $O/accel_native.log
