#!/usr/bin/env python3
"""Run-to-run determinism of the native training step (world 1): the same seed and data must give
bit-identical master weights across two eager runs and between the graph-captured and eager paths.
  python tools/determinism_check.py [--model resnet18] [--batch 16] [--hw 32] [--steps 4] [--optim sgd|lars|adamw]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dbx_distributed_pytorch_examples_amd.engine.native_trainer import NativeTrainer, OptimConfig  # noqa: E402
from dbx_distributed_pytorch_examples_amd.models import build_model  # noqa: E402


def run(a, use_graphs):
    torch.manual_seed(0)
    m = build_model(a.model, num_classes=10)
    lr = {"sgd": 0.05, "lars": 2.0, "adamw": 1e-3}[a.optim]
    tr = NativeTrainer(m, a.batch, (a.hw, a.hw), torch.device("cuda:0"), optim=OptimConfig(name=a.optim, lr=lr),
                       use_graphs=use_graphs)
    w0 = tr.prog.master.detach().clone()
    g = torch.Generator().manual_seed(100)
    for _ in range(a.steps):
        img = torch.randint(0, 256, (a.batch, a.hw, a.hw, 3), dtype=torch.uint8, generator=g)
        lab = torch.randint(0, 10, (a.batch,), generator=g)
        tr.step(img.cuda(), lab.cuda())
    torch.cuda.synchronize()
    return w0, tr.prog.master.detach().clone()


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--model", default="resnet18")
    p.add_argument("--batch", type=int, default=16)
    p.add_argument("--hw", type=int, default=32)
    p.add_argument("--steps", type=int, default=4)
    p.add_argument("--optim", default="sgd", choices=["sgd", "lars", "adamw"])
    p.add_argument("--strict", action="store_true", help="fail unless bit-identical")
    a = p.parse_args()
    w0, e1 = run(a, False)
    _, e2 = run(a, False)
    _, g1 = run(a, True)
    upd = (e1 - w0).norm()
    res = {k: ((x - e1).norm() / upd).item() for k, x in (("eager_vs_eager", e2), ("graph_vs_eager", g1))}
    exact = {k: bool(torch.equal(x, e1)) for k, x in (("eager_vs_eager", e2), ("graph_vs_eager", g1))}
    print(f"determinism {a.model} {a.optim} b{a.batch} {a.hw}px {a.steps} steps: update-relative diff {res} bit-exact {exact}",
          flush=True)
    if a.strict and not all(exact.values()):
        sys.exit(1)


if __name__ == "__main__":
    main()
