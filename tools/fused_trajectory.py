#!/usr/bin/env python3
"""Training-loss trajectories of the native engine with the fused kernel paths on vs off (same init,
data and SGD schedule; ResNet-50 at 224 so the fused conv3 backward and the patch kernels are in use)
next to eager torch autocast-bf16. At a stable learning rate the native variants must track each other
and the torch run; at the chaotic learning rates of a short warmup any two stacks diverge.

  python tools/fused_trajectory.py [--steps 60] [--lr 0.02] [--batch 256]
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
ap.add_argument("--classes", type=int, default=100)
ap.add_argument("--size", type=int, default=224)
ap.add_argument("--batch", type=int, default=256)
ap.add_argument("--steps", type=int, default=60)
ap.add_argument("--lr", type=float, default=0.02)
ap.add_argument("--noise", type=float, default=48.0)
a = ap.parse_args()
dev = torch.device("cuda")
x, y = learnable_synthetic(a.batch * a.steps, a.size, a.classes, seed=1, device=dev, noise=a.noise)
torch.manual_seed(0)
base = build_model("resnet50", num_classes=a.classes)
MEAN = torch.tensor((0.485, 0.456, 0.406), device=dev).view(1, 3, 1, 1) * 255
STD = torch.tensor((0.229, 0.224, 0.225), device=dev).view(1, 3, 1, 1) * 255
VARIANTS = {"native fused": {"DBX_ENGINE": "fuse_dw=1"},
            "native unfused": {"DBX_ENGINE": "fuse_dw=0,stem_wgrad=generic"}}
curves = {}
for name, env in VARIANTS.items():
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    tr = NativeTrainer(copy.deepcopy(base), a.batch, (a.size, a.size), dev,
                       optim=OptimConfig(lr=a.lr, momentum=0.9, weight_decay=5e-5))
    ls = []
    for s in range(a.steps):
        tr.step(x[s * a.batch:(s + 1) * a.batch], y[s * a.batch:(s + 1) * a.batch])
        loss, _ = tr.read_metrics()
        ls.append(loss / a.batch)
    curves[name] = ls
    for k, v in old.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    del tr
    torch.cuda.empty_cache()
m = copy.deepcopy(base).to(dev).to(memory_format=torch.channels_last)
opt = torch.optim.SGD(m.parameters(), lr=a.lr, momentum=0.9, weight_decay=5e-5)
ls = []
for s in range(a.steps):
    xb = x[s * a.batch:(s + 1) * a.batch].permute(0, 3, 1, 2).float()
    xb = ((xb - MEAN) / STD).contiguous(memory_format=torch.channels_last)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        loss = F.cross_entropy(m(xb), y[s * a.batch:(s + 1) * a.batch])
    opt.zero_grad(set_to_none=True)
    loss.backward()
    opt.step()
    ls.append(loss.item())
curves["torch autocast bf16"] = ls
names = list(curves)
print(f"ResNet-50 {a.size}x{a.size} b{a.batch} lr {a.lr} (SGD m0.9, no warmup), {a.classes} classes")
print("step " + " ".join(f"{n:>22s}" for n in names))
for s in range(0, a.steps, max(1, a.steps // 20)):
    print(f"{s:4d} " + " ".join(f"{curves[n][s]:22.4f}" for n in names))
for n in names:
    tail = curves[n][-10:]
    print(f"mean loss of the last 10 steps, {n}: {sum(tail) / len(tail):.4f}")
