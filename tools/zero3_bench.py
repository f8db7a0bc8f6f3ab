#!/usr/bin/env python3
"""Autograd-engine ResNet-50 throughput on one GPU: flat-bucket DDP vs ZeRO-3 (parallel/fsdp.py) vs
ZeRO-3 with CPU offload. At world size 1 a shard is the whole model, so this isolates the cost of the
per-block gather / release / pack / optimizer-on-shards machinery (and of the host step for offload)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dbx_distributed_pytorch_examples_amd.config import OptimizerConfig  # noqa: E402
from dbx_distributed_pytorch_examples_amd.engine.autograd_trainer import AutogradTrainer  # noqa: E402
from dbx_distributed_pytorch_examples_amd.models import build_model  # noqa: E402


def run(stage, offload, batch=128, steps=10, warmup=3):
    torch.manual_seed(0)
    dev = torch.device("cuda:0")
    tr = AutogradTrainer(build_model("resnet50", num_classes=1000), dev,
                         OptimizerConfig(name="adamw", lr=2e-4, weight_decay=0.01), zero_stage=stage,
                         offload_optimizer=offload, offload_param=offload)
    x = torch.randn(batch, 3, 224, 224, device=dev)
    y = torch.randint(0, 1000, (batch,), device=dev)
    for _ in range(warmup):
        tr.step(x, y)
    torch.cuda.synchronize()
    torch.cuda.reset_peak_memory_stats()
    t0 = time.perf_counter()
    for _ in range(steps):
        tr.step(x, y)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    out = {"zero_stage": stage, "offload": offload, "batch": batch, "img_per_s": round(batch * steps / dt, 1),
           "ms_per_step": round(1000 * dt / steps, 2), "peak_mem_gib": round(torch.cuda.max_memory_allocated() / 2**30, 2)}
    del tr
    torch.cuda.empty_cache()
    return out


if __name__ == "__main__":
    for stage, off in ((0, False), (3, False), (3, True)):
        print(json.dumps(run(stage, off)), flush=True)
