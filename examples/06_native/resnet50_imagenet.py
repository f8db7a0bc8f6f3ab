#!/usr/bin/env python3
"""The framework's flagship path: ResNet-50 on the native engine (NHWC bf16 HIP kernels,
graph-captured step, flat-bucket DDP over RCCL), driven by a YAML config.

    python -m dbx_distributed_pytorch_examples_amd.launch --nproc-per-node 8 \\
        examples/06_native/resnet50_imagenet.py configs/resnet50_imagenet_8192.yaml
    python examples/06_native/resnet50_imagenet.py configs/resnet50_imagenet_synthetic.yaml max_steps=20
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from dbx_distributed_pytorch_examples_amd.train.cli import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main())
