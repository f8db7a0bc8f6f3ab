#!/bin/bash
# Composer frontend on engine.native_module: GPU tests (composer + native_module), the Composer example
# with the native route (default) and with DBX_COMPOSER_NATIVE=0.
set -o pipefail
O=gpurun_out/r2s5_composer
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_program_gpu.py -x -q -k "composer or native_module" --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { echo "tests FAILED"; tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 240 python -u examples/03_composer/01_cifar_composer.py --procs 1 --samples 2048 --batch-size 128 --out /tmp/ex > $O/composer_native.log 2>&1 || { echo "composer native FAILED"; tail -20 $O/composer_native.log; exit 1; }
echo "native: $(grep -v amdgpu.ids $O/composer_native.log | tail -3 | tr '\n' ' ' | cut -c1-300)"
DBX_COMPOSER_NATIVE=0 timeout -k 10 240 python -u examples/03_composer/01_cifar_composer.py --procs 1 --samples 2048 --batch-size 128 --out /tmp/ex > $O/composer_torch.log 2>&1 || { echo "composer torch FAILED"; tail -20 $O/composer_torch.log; exit 1; }
echo "torch: $(grep -v amdgpu.ids $O/composer_torch.log | tail -3 | tr '\n' ' ' | cut -c1-300)"
