#!/usr/bin/env python3
"""Per-layer gradient parity of the native ResNet-50 step at 224x224 with the patch kernels
(csrc/conv_patch3.hip: 3x3 fwd / dgrad / wgrad of the 64-channel stage, stem) on vs off, and of
both against fp32 autograd.  python tools/patch_parity.py [--batch 4]"""
import argparse
import copy
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dbx_distributed_pytorch_examples_amd.engine.native_trainer import NativeTrainer, OptimConfig  # noqa: E402
from dbx_distributed_pytorch_examples_amd.models import build_model  # noqa: E402
from dbx_distributed_pytorch_examples_amd.ops import kernels as K  # noqa: E402


def run(model, batch, img, lab, patch: bool):
    os.environ["DBX_ENGINE"] = f"patch3={'all' if patch else '0'},stem_patch={int(patch)}"
    m = copy.deepcopy(model)
    tr = NativeTrainer(m, batch, (224, 224), torch.device("cuda"),
                       optim=OptimConfig(lr=0.0, momentum=0.0, weight_decay=0.0), use_graphs=False)
    tr.step(img, lab)
    torch.cuda.synchronize()
    p = tr.prog
    grads = {}
    for name, off, n in p.param_ranges:
        grads[name] = p.grad[off:off + n].clone()
    return p.metrics[0].item() / batch, grads, p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4)
    a = ap.parse_args()
    torch.manual_seed(0)
    model = build_model("resnet50", num_classes=100)
    for n_, m_ in model.named_modules():
        if n_.endswith("bn3"):
            torch.nn.init.constant_(m_.weight, 0.2)
    g = torch.Generator().manual_seed(1)
    img = torch.randint(0, 256, (a.batch, 224, 224, 3), dtype=torch.uint8, generator=g).cuda()
    lab = torch.randint(0, 100, (a.batch,), generator=g).cuda()
    l_on, g_on, p = run(model, a.batch, img, lab, True)
    l_off, g_off, _ = run(model, a.batch, img, lab, False)
    ref = copy.deepcopy(model).cuda().train()
    x = p.x4[..., :3].float().permute(0, 3, 1, 2).contiguous()
    loss = F.cross_entropy(ref(x), lab)
    loss.backward()
    print(f"loss patch {l_on:.5f} implicit {l_off:.5f} fp32 {loss.item():.5f}")
    named = dict(ref.named_parameters())
    worst = []
    for name in g_on:
        a_, b_ = g_on[name].float(), g_off[name].float()
        rg = named[name].grad if name in named else None
        if rg is None:
            continue
        rg = (rg.permute(0, 2, 3, 1) if rg.dim() == 4 else rg).reshape(-1).float()
        d = ((a_ - b_).norm() / (b_.norm() + 1e-20)).item()
        cos_on = (a_ @ rg / (a_.norm() * rg.norm() + 1e-20)).item()
        cos_off = (b_ @ rg / (b_.norm() * rg.norm() + 1e-20)).item()
        worst.append((d, name, cos_on, cos_off))
    worst.sort(reverse=True)
    for d, name, c1, c2 in worst[:15]:
        print(f"{name:40s} on-vs-off relerr {d:.2e}  cos(on,fp32) {c1:.4f}  cos(off,fp32) {c2:.4f}")


if __name__ == "__main__":
    main()
