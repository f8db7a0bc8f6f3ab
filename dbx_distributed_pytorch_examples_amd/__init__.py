"""dbx_distributed_pytorch_examples_amd — MI355X-native distributed image-classification training.

A from-scratch re-design of alexxx-db/dbx-distributed-pytorch-examples for AMD Instinct
MI355X (gfx950): NHWC bf16 ResNet programs on hand-written HIP/CDNA4 kernels, one process per
GPU over RCCL/xGMI, one launcher in place of the reference's five launcher shims.
"""
__version__ = "0.1.0"
