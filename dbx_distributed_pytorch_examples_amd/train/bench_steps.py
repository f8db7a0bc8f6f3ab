"""Step builders for ``bench.py`` (one callable == one full training step)."""
from __future__ import annotations

from typing import Callable, Dict, Tuple

import torch
import torch.nn.functional as F

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def synthetic_uint8_batch(batch: int, size: int, num_classes: int, device, seed: int = 0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randint(0, 256, (batch, size, size, 3), dtype=torch.uint8, generator=g)
    y = torch.randint(0, num_classes, (batch,), dtype=torch.int64, generator=g)
    return x.to(device), y.to(device)


def build_torch_step(args, info) -> Tuple[Callable[[], None], Dict]:
    """Reference-equivalent: stock eager nn.Module + autocast bf16 + torch DDP (RCCL)."""
    from ..models import build_model
    dev = info.device
    model = build_model(args.model, num_classes=args.num_classes).to(dev)
    mf = torch.channels_last if args.channels_last else torch.contiguous_format
    model = model.to(memory_format=mf)
    if info.world_size > 1:
        model = torch.nn.parallel.DistributedDataParallel(model, device_ids=[dev.index],
                                                          bucket_cap_mb=25, gradient_as_bucket_view=True)
    if getattr(args, "optim", "sgd") == "adamw":
        opt = torch.optim.AdamW(model.parameters(), lr=args.lr, weight_decay=0.01)
    elif getattr(args, "optim", "sgd") == "lars":
        from ..engine.autograd_trainer import LARS
        opt = LARS(model.parameters(), lr=args.lr, momentum=0.9, weight_decay=5e-5, trust_coefficient=0.001)
    else:
        opt = torch.optim.SGD(model.parameters(), lr=args.lr, momentum=0.9, weight_decay=5e-5)
    x8, y = synthetic_uint8_batch(args.batch, args.image_size, args.num_classes, dev, seed=info.rank)
    mean = torch.tensor(IMAGENET_MEAN, device=dev).view(1, 3, 1, 1) * 255.0
    std = torch.tensor(IMAGENET_STD, device=dev).view(1, 3, 1, 1) * 255.0

    def step():
        x = x8.permute(0, 3, 1, 2).float().sub_(mean).div_(std).contiguous(memory_format=mf)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = model(x)
            loss = F.cross_entropy(out, y)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()

    step.model = model  # bench.py replica check
    return step, {"memory_format": "channels_last" if args.channels_last else "nchw",
                  "ddp": "torch DDP 25MiB buckets" if info.world_size > 1 else "none"}


def build_step(args, info):
    if args.impl == "torch":
        return build_torch_step(args, info)
    from .native_step import build_native_step
    return build_native_step(args, info)
