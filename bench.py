#!/usr/bin/env python3
"""Headline benchmark: ResNet-50 ImageNet-1K (224x224, 1000 classes) training throughput.

Metric (BASELINE.json): images/sec for the whole job, ResNet-50 ImageNet-1K, at 1/2/4/8
MI355X, bf16, synthetic data + random-init weights, weak scaling (fixed per-GPU batch).

  python bench.py --gpus N --steps K --warmup W        # N=1 runs in-process
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Implementations (``--impl``):
  native  the framework's flagship path: NHWC bf16 ResNet program on the hand-written HIP
          kernels (dbx.ops), graph-captured step, flat-bucket DDP on RCCL (default)
  torch   reference-equivalent stock PyTorch-ROCm: eager nn.Module, autocast bf16,
          torch DDP on RCCL, torch.optim.SGD — the measured "reference" column of BASELINE.md

Every timed step does the full work: input normalisation from uint8, forward, loss,
backward, gradient all-reduce (N>1) and the SGD-momentum update.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

# Reference-equivalent stock PyTorch ResNet-50 throughput on ONE MI355X, measured with
# `python bench.py --impl torch --batch B` (eager nn.Module, channels_last, autocast bf16, MIOpen
# convs, torch.optim.SGD; BASELINE.md, profiles/r1_torch_reference/). Keyed by per-GPU batch.
BASELINE_IMG_PER_SEC_PER_GPU = {256: 5941.96, 1024: 6496.62}

# BASELINE.json's other configs (the headline default is ResNet-50 ImageNet-1K, 1024/GPU).
PRESETS = {
    "resnet18_cifar10": dict(model="resnet18", image_size=32, num_classes=10, batch=256),
    "resnet50_tiny_imagenet": dict(model="resnet50", image_size=64, num_classes=200, batch=512),
    "resnet50_imagenet_zero1": dict(model="resnet50", image_size=224, num_classes=1000, batch=256, optim="adamw",
                                    zero=1),
    "resnet50_imagenet_8192": dict(model="resnet50", image_size=224, num_classes=1000, batch=1024),
}


def parse_args(argv=None):
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=30)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--batch", type=int, default=1024,
                   help="per-GPU batch (weak scaling); 1024 x 8 GPUs = the 8192 large-batch north-star config")
    p.add_argument("--impl", default="native", choices=["native", "torch"])
    p.add_argument("--model", default="resnet50")
    p.add_argument("--image-size", type=int, default=224)
    p.add_argument("--num-classes", type=int, default=1000)
    p.add_argument("--channels-last", type=int, default=1, help="torch impl only")
    p.add_argument("--lr", type=float, default=None, help="default: 0.1 (sgd) / 2e-4 (adamw)")
    p.add_argument("--optim", default="sgd", choices=["sgd", "adamw", "lars"])
    p.add_argument("--zero", type=int, default=0, choices=[0, 1, 2], help="native impl: ZeRO stage")
    p.add_argument("--preset", default="", choices=[""] + sorted(PRESETS),
                   help="one of BASELINE.json's other configs (sets model/size/classes/batch/optim)")
    p.add_argument("--json-out", default=None)
    a = p.parse_args(argv)
    for k, v in PRESETS.get(a.preset, {}).items():
        setattr(a, k, v)
    if a.lr is None:
        a.lr = {"sgd": 0.1, "lars": 9.0}.get(a.optim, 2e-4)
    return a


def main(argv=None) -> int:
    args = parse_args(argv)
    from dbx_distributed_pytorch_examples_amd.parallel import dist as ddist
    from dbx_distributed_pytorch_examples_amd.train.bench_steps import build_step

    info = ddist.init_distributed()
    if info.world_size != args.gpus and info.rank == 0:
        print(f"[bench] warning: --gpus {args.gpus} but WORLD_SIZE={info.world_size}", file=sys.stderr)
    torch.manual_seed(1234 + info.rank)
    step, meta = build_step(args, info)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    ddist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    ddist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    elapsed = ddist.all_reduce_max(elapsed)

    n = info.world_size
    imgs = args.batch * n * args.steps
    value = imgs / elapsed
    headline = args.model == "resnet50" and args.image_size == 224 and args.num_classes == 1000 and args.optim == "sgd"
    base = BASELINE_IMG_PER_SEC_PER_GPU.get(args.batch) if headline else None
    out = {
        "metric": "images/sec (whole node) ResNet-50 ImageNet-1K at 1/2/4/8 MI355X; top-1 acc",
        "value": round(value, 2),
        "unit": "images/s",
        "n_gpus": n,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1000.0 * elapsed / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": (round(value / (base * n), 4) if base else None),
        "dtype": "bf16",
        "data": f"synthetic (uint8 NHWC {args.image_size}x{args.image_size} images + random labels, on-device; "
                "random-init weights)",
        "config": {
            "model": f"{args.model} ImageNet-1K {args.image_size}x{args.image_size} {args.num_classes} classes"
                     + (" large-batch (global 8192 at 8 GPUs)" if args.batch == 1024 else ""),
            "global_batch": args.batch * n,
            "per_gpu_batch": args.batch,
            "seq_len": None,
            "parallelism": f"dp{n}",
            "impl": args.impl,
            "optimizer": {"sgd": "SGD momentum 0.9 nesterov=False wd 5e-5",
                          "lars": "LARS (eta 1e-3) + SGD momentum 0.9 wd 5e-5"}.get(args.optim, "AdamW wd 0.01")
                         + (f", ZeRO-{args.zero}" if args.zero else ""),
            **meta,
        },
    }
    if info.rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    ddist.destroy()
    return 0


if __name__ == "__main__":
    sys.exit(main())
