#!/bin/bash
# Every reference-notebook example on ONE GPU (one process, small synthetic splits): the GPU paths of the
# examples, which the CPU test suite only covers with --cpu. A Python failure of one example is reported and
# the next one runs; a fault / abort / time limit (124, 134, 137, 139) ends the script there.
set -o pipefail
O=gpurun_out/r2s5_examples_all
mkdir -p $O
fails=0
run() {
  local name=$1; shift
  timeout -k 10 240 "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -v amdgpu.ids $O/$name.log | tail -1 | cut -c1-150)"
  if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  [ $rc -ne 0 ] && fails=$((fails+1))
  return 0
}
E=examples
run mnist python -u $E/01_torch_distributor/01_basic_mnist.py --procs 1 --samples 512 --out /tmp/ex
run td_cifar python -u $E/01_torch_distributor/02_cifar_resnet.py --procs 1 --samples 512 --out /tmp/ex
run td_tiny python -u $E/01_torch_distributor/03_tiny_imagenet_resnet.py --procs 1 --samples 512 --out /tmp/ex
run td_tiny_mds python -u $E/01_torch_distributor/03a_tiny_imagenet_mds.py --procs 1 --samples 512 --out /tmp/ex
run ds_cifar python -u $E/02_deepspeed/01_cifar_deepspeed.py --procs 1 --samples 512 --out /tmp/ex
run ds_tiny python -u $E/02_deepspeed/02_tiny_imagenet_deepspeed.py --procs 1 --samples 512 --out /tmp/ex
run ds_1k python -u $E/02_deepspeed/03_imagenet_1k_deepspeed.py --procs 1 --samples 256 --out /tmp/ex
run composer python -u $E/03_composer/01_cifar_composer.py --procs 1 --samples 512 --out /tmp/ex
run accelerate python -u $E/04_accelerate/01_cifar_accelerate.py --samples 1024 --batch-size 128 --out /tmp/ex
run accelerate_native python -u $E/04_accelerate/01_cifar_accelerate.py --native --samples 1024 --batch-size 128 --out /tmp/ex
run ray_fmnist python -u $E/05_ray/01_fashion_mnist_ray.py --procs 1 --samples 512 --out /tmp/ex
run ray_cifar python -u $E/05_ray/02_cifar_ray.py --procs 1 --samples 512 --out /tmp/ex
run ray_cifar_native python -u $E/05_ray/02_cifar_ray.py --native --procs 1 --samples 1024 --batch-size 128 --out /tmp/ex
run native python -u $E/06_native/resnet50_imagenet.py configs/resnet50_imagenet_synthetic.yaml max_steps=10
echo "examples failed: $fails"
