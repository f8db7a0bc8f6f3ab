#!/usr/bin/env python3
"""Throughput of the reference's DOMINANT workload: frozen-backbone ResNet + new head.

Every TorchDistributor / DeepSpeed ResNet notebook of the reference trains only
``fc = Sequential(Dropout(0.5), Linear(in, C))`` on a frozen ImageNet backbone:
ResNet-18 / CIFAR-10 32x32 b256 Adam 1e-3 (`01_torch_distributor/02_cifar_torch_distributor_resnet.py:141-213`),
ResNet-50 / TinyImageNet 64x64 b256 (`03_tiny_imagenet_torch_distributor_resnet.py:125-197`) and b512 (03a, MDS),
ResNet-50 / ImageNet-1K 224x224 b32 Adam 1e-5 (`02_deepspeed/03_1k_imagenet_deepspeed_resnet.py:121-186`).

  native     engine/frozen_trainer.FrozenFeatureTrainer: the backbone as the native NHWC program in
             inference mode (BN folded, no activations kept), the head stepped by autograd
  reference  what the notebooks run: the whole model in train() mode under autocast bf16
             (channels_last), cross-entropy, backward (reaches the head only), torch.optim.Adam

Synthetic uint8 images + random labels on the device, random-init backbone. One JSON line per
(config, impl): images/s over --steps timed steps after --warmup.

  python tools/bench_frozen.py [--steps 30] [--warmup 5] [--configs r18_cifar,r50_tiny,...]
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dbx_distributed_pytorch_examples_amd.config import OptimizerConfig  # noqa: E402
from dbx_distributed_pytorch_examples_amd.models.wrappers import FrozenBackboneClassifier  # noqa: E402

CONFIGS = {
    # name: (arch, image size, classes, batch, Adam lr, reference file)
    "r18_cifar": ("resnet18", 32, 10, 256, 1e-3, "01_torch_distributor/02_cifar_torch_distributor_resnet.py"),
    "r50_tiny": ("resnet50", 64, 200, 256, 1e-3, "01_torch_distributor/03_tiny_imagenet_torch_distributor_resnet.py"),
    "r50_tiny_mds": ("resnet50", 64, 200, 512, 1e-3, "01_torch_distributor/03a_tiny_imagenet_..._mds.py"),
    "r50_imagenet_b32": ("resnet50", 224, 1000, 32, 1e-5, "02_deepspeed/03_1k_imagenet_deepspeed_resnet.py"),
    "r50_imagenet_b256": ("resnet50", 224, 1000, 256, 1e-5, "(03_1k at a GPU-filling batch)"),
}
MEAN = (0.485, 0.456, 0.406)
STD = (0.229, 0.224, 0.225)


def timed(step, steps, warmup):
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    return time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--configs", default=",".join(CONFIGS))
    ap.add_argument("--impls", default="native,reference")
    a = ap.parse_args()
    dev = torch.device("cuda")
    for name in a.configs.split(","):
        arch, s, nc, b, lr, ref = CONFIGS[name]
        torch.manual_seed(0)
        x8 = torch.randint(0, 256, (b, s, s, 3), dtype=torch.uint8, device=dev)
        y = torch.randint(0, nc, (b,), device=dev)
        for impl in a.impls.split(","):
            model = FrozenBackboneClassifier(arch, num_classes=nc)
            if impl == "native":
                from dbx_distributed_pytorch_examples_amd.engine.frozen_trainer import FrozenFeatureTrainer
                tr = FrozenFeatureTrainer(model, b, (s, s), dev, OptimizerConfig(name="adam", lr=lr))

                def step():
                    tr.step(x8, y)
            else:
                model = model.to(dev).to(memory_format=torch.channels_last).train()
                opt = torch.optim.Adam([p for p in model.parameters() if p.requires_grad], lr=lr)
                mean = torch.tensor(MEAN, device=dev).view(1, 3, 1, 1) * 255.0
                std = torch.tensor(STD, device=dev).view(1, 3, 1, 1) * 255.0

                def step():
                    xin = x8.permute(0, 3, 1, 2).float().sub_(mean).div_(std).contiguous(
                        memory_format=torch.channels_last)
                    with torch.autocast("cuda", dtype=torch.bfloat16):
                        loss = F.cross_entropy(model(xin), y)
                    opt.zero_grad(set_to_none=True)
                    loss.backward()
                    opt.step()
            el = timed(step, a.steps, a.warmup)
            print(json.dumps({"config": name, "impl": impl, "model": arch, "image_size": s, "classes": nc,
                              "batch": b, "images_per_s": round(b * a.steps / el, 1),
                              "ms_per_step": round(1000 * el / a.steps, 3), "reference": ref}), flush=True)
            del model
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
