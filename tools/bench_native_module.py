#!/usr/bin/env python3
"""A user-written training loop (the Accelerate / Ray notebooks' shape: ``logits = model(x); loss =
criterion(logits, y); loss.backward(); optimizer.step()``) on the stock torch module vs the same loop
on ``engine.native_module`` (native HIP forward / backward through autograd).

  torch   channels_last model under autocast bf16 (what Accelerate's mixed_precision="bf16" runs)
  native  native_module(model, batch, hw): float NCHW input, bf16 HIP program, fp32 torch loss
  prepare the notebook's own call with no flags: ``Accelerator().prepare(model, optimizer)`` (Ray config:
          ``ray.train.torch.prepare_model(model)``) -- the frontends put the ResNet on the native
          program by default (compiled for the first batch), the optimizer built before prepare

Synthetic normalised float inputs + random labels on the device; one JSON line per (config, impl).
  python tools/bench_native_module.py [--steps 20] [--warmup 5]
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dbx_distributed_pytorch_examples_amd.engine.native_module import native_module  # noqa: E402
from dbx_distributed_pytorch_examples_amd.models import build_model  # noqa: E402

CONFIGS = {
    # name: (arch, size, classes, batch, optimizer, reference)
    "accelerate_r50_cifar": ("resnet50", 32, 10, 128, "adam", "04_accelerate/01_cifar_accelerate.ipynb (Adam 1e-3, wd 1e-4)"),
    "ray_r18_cifar": ("resnet18", 32, 10, 256, "adam", "05_ray/02_cifar_resnet_pytorch_ray.ipynb (Adam 1e-5)"),
    "composer_r50_cifar": ("resnet50", 32, 1000, 128, "adam", "03_composer/01_cifar_composer_resnet.ipynb (1000-way head)"),
    "r50_imagenet_b256": ("resnet50", 224, 1000, 256, "sgd", "ImageNet-1K loop at a GPU-filling batch"),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--configs", default=",".join(CONFIGS))
    ap.add_argument("--impls", default="torch,native,prepare")
    a = ap.parse_args()
    dev = torch.device("cuda")
    for name in a.configs.split(","):
        arch, s, nc, b, opt_name, ref = CONFIGS[name]
        x = torch.randn(b, 3, s, s, device=dev)
        y = torch.randint(0, nc, (b,), device=dev)
        for impl in a.impls.split(","):
            torch.manual_seed(0)
            model = build_model(arch, num_classes=nc)
            acc = None
            if impl == "native":
                model = native_module(model, b, (s, s), dev).train()
                xin = x
            elif impl == "prepare":
                from dbx_distributed_pytorch_examples_amd.frontends.accelerate import Accelerator
                from dbx_distributed_pytorch_examples_amd.frontends.ray import prepare_model
                opt0 = (torch.optim.Adam(model.parameters(), lr=1e-3, weight_decay=1e-4) if opt_name == "adam"
                        else torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5))
                if name.startswith("ray"):
                    model = prepare_model(model).train()
                else:
                    acc = Accelerator(mixed_precision="bf16")
                    model, opt0 = acc.prepare(model, opt0)
                    model.train()
                xin = x
            else:
                model = model.to(dev).to(memory_format=torch.channels_last).train()
                xin = x.contiguous(memory_format=torch.channels_last)
            if impl == "prepare":
                opt = opt0  # built before prepare, as the notebooks do
            else:
                opt = (torch.optim.Adam(model.parameters(), lr=1e-3, weight_decay=1e-4) if opt_name == "adam"
                       else torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5))

            def step():
                opt.zero_grad(set_to_none=True)
                with torch.autocast("cuda", dtype=torch.bfloat16, enabled=(impl == "torch")):
                    loss = F.cross_entropy(model(xin), y, label_smoothing=0.1)
                if acc is not None:
                    acc.backward(loss)
                else:
                    loss.backward()
                opt.step()
            for _ in range(a.warmup):
                step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                step()
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            print(json.dumps({"config": name, "impl": impl, "model": arch, "image_size": s, "batch": b,
                              "images_per_s": round(b * a.steps / el, 1), "ms_per_step": round(1000 * el / a.steps, 3),
                              "reference": ref}), flush=True)
            del model, opt
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
