#!/usr/bin/env python3
"""Step-by-step training-loss trajectory: native engine vs eager torch (autocast bf16 and fp32) on
the same init, data and SGD schedule. Bisects training-quality differences between the stacks.

  python tools/trajectory_parity.py [--model resnet50] [--size 64] [--steps 40] [--lr 0.1]
"""
import argparse
import copy
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dbx_distributed_pytorch_examples_amd.data.datasets import learnable_synthetic  # noqa: E402
from dbx_distributed_pytorch_examples_amd.engine.native_trainer import NativeTrainer, OptimConfig  # noqa: E402
from dbx_distributed_pytorch_examples_amd.models import build_model  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="resnet50")
ap.add_argument("--classes", type=int, default=100)
ap.add_argument("--size", type=int, default=64)
ap.add_argument("--batch", type=int, default=256)
ap.add_argument("--steps", type=int, default=40)
ap.add_argument("--lr", type=float, default=0.1)
ap.add_argument("--graphs", type=int, default=1)
a = ap.parse_args()
dev = torch.device("cuda")
x, y = learnable_synthetic(a.batch * a.steps, a.size, a.classes, seed=1, device=dev)
torch.manual_seed(0)
base = build_model(a.model, num_classes=a.classes)
r16 = copy.deepcopy(base).to(dev).to(memory_format=torch.channels_last)
r32 = copy.deepcopy(base).to(dev).to(memory_format=torch.channels_last)
nat = NativeTrainer(base, a.batch, (a.size, a.size), dev, optim=OptimConfig(lr=a.lr, weight_decay=5e-5),
                    use_graphs=bool(a.graphs))
o16 = torch.optim.SGD(r16.parameters(), lr=a.lr, momentum=0.9, weight_decay=5e-5)
o32 = torch.optim.SGD(r32.parameters(), lr=a.lr, momentum=0.9, weight_decay=5e-5)
mean = torch.tensor((0.485, 0.456, 0.406), device=dev).view(1, 3, 1, 1) * 255.0
std = torch.tensor((0.229, 0.224, 0.225), device=dev).view(1, 3, 1, 1) * 255.0
print("step native ref_bf16 ref_fp32")
for s in range(a.steps):
    xb, yb = x[s * a.batch:(s + 1) * a.batch], y[s * a.batch:(s + 1) * a.batch]
    nat.step(xb, yb)
    ln, _ = nat.read_metrics()
    xi = xb.permute(0, 3, 1, 2).float().sub_(mean).div_(std).contiguous(memory_format=torch.channels_last)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        l16 = F.cross_entropy(r16(xi), yb)
    o16.zero_grad(set_to_none=True)
    l16.backward()
    o16.step()
    l32 = F.cross_entropy(r32(xi), yb)
    o32.zero_grad(set_to_none=True)
    l32.backward()
    o32.step()
    print(f"{s:3d} {ln / a.batch:8.4f} {l16.item():8.4f} {l32.item():8.4f}", flush=True)
