"""bench.py step builder for the native (HIP-kernel, graph-captured) ResNet path."""
from __future__ import annotations

import os

import torch

from ..engine.native_trainer import NativeTrainer, OptimConfig
from ..models import build_model


def build_native_step(args, info):
    dev = info.device
    torch.manual_seed(0)  # identical init on every rank (DDP also broadcasts from rank 0)
    model = build_model(args.model, num_classes=args.num_classes)
    if getattr(args, "optim", "sgd") == "adamw":
        opt = OptimConfig(name="adamw", lr=args.lr, weight_decay=0.01)
    elif getattr(args, "optim", "sgd") == "lars":
        opt = OptimConfig(name="lars", lr=args.lr, momentum=0.9, weight_decay=5e-5, trust_coefficient=0.001)
    else:
        opt = OptimConfig(name="sgd", lr=args.lr, momentum=0.9, weight_decay=5e-5)
    use_graphs = os.environ.get("DBX_GRAPHS", "1") == "1"
    ar_dtype = torch.bfloat16 if os.environ.get("DBX_ALLREDUCE_BF16", "0") == "1" else torch.float32
    tr = NativeTrainer(model, args.batch, (args.image_size, args.image_size), dev, optim=opt,
                       use_graphs=use_graphs, allreduce_dtype=ar_dtype, zero_stage=getattr(args, "zero", 0))
    g = torch.Generator(device="cpu").manual_seed(1000 + info.rank)
    img = torch.randint(0, 256, (args.batch, args.image_size, args.image_size, 3), dtype=torch.uint8, generator=g)
    lab = torch.randint(0, args.num_classes, (args.batch,), dtype=torch.int64, generator=g)
    tr.prog.img_u8.copy_(img)
    tr.prog.labels.copy_(lab)

    def step():
        tr.step()

    extra = {}
    if tr.zero is not None:
        extra["zero"] = (f"ZeRO-{tr.zero.stage}: per-segment fp32 reduce-scatter (overlapped with backward), sharded "
                         f"{opt.name} update, bf16 all-gather; {tr.zero.bytes_per_step / 2**20:.1f} MiB sent/rank/step")
    return step, {**extra, "memory_format": "nhwc", "graphs": use_graphs,
                  "ddp": (f"flat-bucket {'RCCL' if info.backend == 'nccl' else info.backend} all-reduce, "
                          f"{tr.bucket_cap * 4 >> 20} MiB chunks, "
                          f"{str(ar_dtype).split('.')[-1]}, overlapped per backward segment") if tr.world > 1 else "none",
                  "kernels": "dbx HIP (conv implicit-GEMM MFMA + fused BN/ReLU/pool/CE/SGD)"}
