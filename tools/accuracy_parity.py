#!/usr/bin/env python3
"""Top-1 accuracy parity: the native HIP engine vs the reference-equivalent stock PyTorch stack.

Both train the SAME random-init ResNet (identical initial weights, data order, hyper-parameters)
on a learnable synthetic task (``data.datasets.learnable_synthetic``: class prototypes + shifts +
noise; no dataset download) and report held-out top-1 after every epoch. The reference side is
eager torch (channels_last, autocast bf16, torch.optim.SGD) — the same column as BASELINE.md.

  python tools/accuracy_parity.py [--model resnet50] [--classes 100] [--size 64] [--epochs 4]
"""
import argparse
import copy
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dbx_distributed_pytorch_examples_amd.data.datasets import learnable_synthetic  # noqa: E402
from dbx_distributed_pytorch_examples_amd.engine.native_trainer import NativeTrainer, OptimConfig  # noqa: E402
from dbx_distributed_pytorch_examples_amd.models import build_model  # noqa: E402

MEAN = (0.485, 0.456, 0.406)
STD = (0.229, 0.224, 0.225)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--classes", type=int, default=100)
    ap.add_argument("--size", type=int, default=64)
    ap.add_argument("--train", type=int, default=25600)
    ap.add_argument("--val", type=int, default=4096)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--epochs", type=int, default=4)
    ap.add_argument("--lr", type=float, default=0.05)
    ap.add_argument("--warmup-epochs", type=int, default=1)
    ap.add_argument("--noise", type=float, default=48.0, help="pixel noise std (0..255 units): task difficulty")
    ap.add_argument("--json-out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda")
    xtr, ytr = learnable_synthetic(a.train, a.size, a.classes, seed=1, device=dev, noise=a.noise)
    xva, yva = learnable_synthetic(a.val, a.size, a.classes, seed=2, device=dev, noise=a.noise)
    torch.manual_seed(0)
    base = build_model(a.model, num_classes=a.classes)
    ref_model = copy.deepcopy(base).to(dev).to(memory_format=torch.channels_last)
    steps_per_epoch = a.train // a.batch
    total = steps_per_epoch * a.epochs
    warm = steps_per_epoch * a.warmup_epochs

    def lr_at(s):  # linear warmup, then cosine (the usual large-batch ResNet recipe)
        if s < warm:
            return a.lr * (s + 1) / warm
        return a.lr * 0.5 * (1 + torch.cos(torch.tensor((s - warm) / max(1, total - warm) * 3.14159265)).item())

    # native engine
    nat = NativeTrainer(base, a.batch, (a.size, a.size), dev, optim=OptimConfig(lr=a.lr, weight_decay=5e-5))
    # reference-equivalent
    opt = torch.optim.SGD(ref_model.parameters(), lr=a.lr, momentum=0.9, weight_decay=5e-5)
    mean = torch.tensor(MEAN, device=dev).view(1, 3, 1, 1) * 255.0
    std = torch.tensor(STD, device=dev).view(1, 3, 1, 1) * 255.0

    def ref_in(x8):
        return x8.permute(0, 3, 1, 2).float().sub_(mean).div_(std).contiguous(memory_format=torch.channels_last)

    def top1_native():
        correct = 0
        for i in range(0, a.val - a.batch + 1, a.batch):
            out = nat.evaluate_batch(xva[i:i + a.batch], yva[i:i + a.batch])
            correct += (out.float().argmax(1) == yva[i:i + a.batch]).sum().item()
        return correct / (a.val // a.batch * a.batch)

    @torch.no_grad()
    def top1_torch_eval_of_native():
        """native weights + running statistics evaluated by a stock torch module (cross-check)"""
        m = copy.deepcopy(ref_model)
        m.load_state_dict({k: v.detach().clone() for k, v in base.state_dict().items()})
        m.eval()
        correct = 0
        for i in range(0, a.val - a.batch + 1, a.batch):
            with torch.autocast("cuda", dtype=torch.bfloat16):
                out = m(ref_in(xva[i:i + a.batch]))
            correct += (out.float().argmax(1) == yva[i:i + a.batch]).sum().item()
        return correct / (a.val // a.batch * a.batch)

    @torch.no_grad()
    def top1_ref():
        ref_model.eval()
        correct = 0
        for i in range(0, a.val - a.batch + 1, a.batch):
            with torch.autocast("cuda", dtype=torch.bfloat16):
                out = ref_model(ref_in(xva[i:i + a.batch]))
            correct += (out.float().argmax(1) == yva[i:i + a.batch]).sum().item()
        ref_model.train()
        return correct / (a.val // a.batch * a.batch)

    hist = []
    step = 0
    g = torch.Generator(device="cpu").manual_seed(7)
    for ep in range(a.epochs):
        perm = torch.randperm(a.train, generator=g).to(dev)
        t0 = time.time()
        ln = lr_ = 0.0
        lr_sum = 0.0
        rl = 0.0
        for b in range(steps_per_epoch):
            idx = perm[b * a.batch:(b + 1) * a.batch]
            x8, y = xtr[idx], ytr[idx]
            lr = lr_at(step)
            nat.set_lr(lr)
            nat.step(x8, y)
            for pg in opt.param_groups:
                pg["lr"] = lr
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = F.cross_entropy(ref_model(ref_in(x8)), y)
            opt.zero_grad(set_to_none=True)
            loss.backward()
            opt.step()
            rl += loss.detach()
            lr_sum += lr
            step += 1
        nl, _ = nat.read_metrics()
        rec = {"epoch": ep + 1, "native_train_loss": round(nl / (steps_per_epoch * a.batch), 4),
               "reference_train_loss": round(rl.item() / steps_per_epoch, 4),
               "native_top1": top1_native(), "reference_top1": top1_ref(),
               "native_weights_torch_eval_top1": top1_torch_eval_of_native(), "wall_s": round(time.time() - t0, 1)}
        hist.append(rec)
        print(json.dumps(rec), flush=True)
    out = {"model": a.model, "classes": a.classes, "noise": a.noise, "lr": a.lr, "image_size": a.size, "train": a.train, "val": a.val,
           "batch": a.batch, "epochs": a.epochs, "optimizer": f"SGD m0.9 wd5e-5, lr {a.lr}, {a.warmup_epochs} warmup epoch(s) + cosine", "history": hist,
           "data": "learnable synthetic (class prototypes + shift + noise), held-out split"}
    print(json.dumps(out))
    if a.json_out:
        with open(a.json_out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
