"""dbx_distributed_pytorch_examples_amd — MI355X-native distributed image-classification training.

A from-scratch re-design of alexxx-db/dbx-distributed-pytorch-examples for AMD Instinct
MI355X (gfx950): NHWC bf16 ResNet programs on hand-written HIP/CDNA4 kernels, one process per
GPU over RCCL/xGMI, one launcher in place of the reference's five launcher shims.
"""
import os as _os

__version__ = "0.1.0"

# HIP graph launch runs a captured graph's parallel branches on extra queues. With the runtime's
# default queue count, launching the framework's step graphs (main stream + side-stream weight
# gradients / comm-stream buckets) crashed the HIP runtime on the host in hipGraphLaunch for some
# graph shapes and stream assignments (torch's bundled HIP 7.0; a stream-pool walk past its end).
# Two queues -- the main chain plus one for the overlapped branches -- never crashed and keep the
# full overlap throughput (headline 16.46k, CIFAR 252.9k, TinyImageNet 95.5k img/s), one queue
# crashes never either but serializes the branches (-1.2 % / -6.8 % / -7.8 %): profiles/r4_final2/.
# Read by the HIP runtime when it initialises, so set here, before any device use; an explicit
# setting in the environment wins.
_os.environ.setdefault("DEBUG_HIP_FORCE_GRAPH_QUEUES", "2")
