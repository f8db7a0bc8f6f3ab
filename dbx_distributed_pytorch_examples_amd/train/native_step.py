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
    from ..engine_config import EngineConfig
    eng = EngineConfig.current()
    use_graphs = eng.graphs
    ar_dtype = torch.bfloat16 if eng.allreduce_bf16 else torch.float32
    tr = NativeTrainer(model, args.batch, (args.image_size, args.image_size), dev, optim=opt,
                       use_graphs=use_graphs, allreduce_dtype=ar_dtype, zero_stage=getattr(args, "zero", 0))
    extra = {}
    if getattr(args, "data", "synthetic") == "mds":
        step, extra["mds"] = _mds_step(args, info, tr)
    else:
        g = torch.Generator(device="cpu").manual_seed(1000 + info.rank)
        img = torch.randint(0, 256, (args.batch, args.image_size, args.image_size, 3), dtype=torch.uint8, generator=g)
        lab = torch.randint(0, args.num_classes, (args.batch,), dtype=torch.int64, generator=g)
        tr.prog.img_u8.copy_(img)
        tr.prog.labels.copy_(lab)

        def step():
            tr.step()

    step.trainer = tr  # bench.py: replica check, watchdog registration
    if tr.zero is not None:
        extra["zero"] = (f"ZeRO-{tr.zero.stage}: per-segment fp32 reduce-scatter (overlapped with backward), sharded "
                         f"{opt.name} update, bf16 all-gather; " + zero_bytes_label(tr.zero))
    return step, {**extra, "memory_format": "nhwc", "graphs": use_graphs,
                  "ddp": (f"flat-bucket {'RCCL' if info.backend == 'nccl' else info.backend} all-reduce, "
                          f"{tr.bucket_cap * 4 >> 20} MiB chunks, "
                          f"{str(ar_dtype).split('.')[-1]}, overlapped per backward segment"
                          + (" (framework RCCL communicator, whole step one HIP graph, weight-gradient side stream "
                             "with late posts)" if tr.ncomm is not None else " (c10d between per-segment graphs)"))
                  + (f"; collectives: {tr.grad_collectives}" if tr.world > 1 else "")
                  if tr.world > 1 or getattr(tr, "segmented", False) else "none",
                  "kernels": "dbx HIP (conv implicit-GEMM MFMA + fused BN/ReLU/pool/CE/SGD)"}


def zero_bytes_label(z) -> str:
    """Ring bytes per rank and step of the ZeRO exchange: at the run's world, and planned at 8 ranks (the
    north-star node) when the run is smaller, so a one-GPU run does not print a bare 0."""
    here = f"{z.bytes_per_step / 2**20:.1f} MiB sent/rank/step at world {z.world}"
    if z.world >= 8:
        return here
    return here + f" (planned at 8 ranks: {z.planned_bytes(8) / 2**20:.1f} MiB sent/rank/step)"


def _mds_step(args, info, tr):
    """The 03a input path, timed with the step. Every rank writes ``--mds-samples`` synthetic
    images of the config's shape as zstd MDS shards ('pil' + 'int' columns, the reference's
    ``MDSWriter(..., compression='zstd')`` call, `03a_tiny_imagenet_torch_distributor_resnet_mds.py:179-223`)
    into its part of one dataset; rank 0 merges the parts' indexes; then every step takes its batch
    from ``NativeImageLoader`` over the shared ``StreamingDataset`` (deterministic rank partition):
    C++ shard reader -> pinned staging ring -> async H2D on the copy stream -> GPU augment (random
    crop + flip) inside the captured step."""
    import atexit
    import json
    import os
    import shutil
    import tempfile
    import time

    import numpy as np
    from PIL import Image

    from ..data.loader import AugmentSpec, NativeImageLoader
    from ..data.mds import MDSWriter, StreamingDataset
    from ..parallel import dist as ddist
    s, B = args.image_size, args.batch
    # a fixed pool (the loader re-iterates epochs): 8 batches per rank, not (steps + warmup) batches
    n = args.mds_samples or 8 * B
    free = shutil.disk_usage(tempfile.gettempdir()).free
    est = n * (s * s * 3 + 64)  # zstd of random pixels does not compress
    if est * info.local_world_size > 0.8 * free:
        raise SystemExit(f"--data mds: ~{est * info.local_world_size / 2**30:.1f} GiB of shards would not fit the "
                         f"{free / 2**30:.1f} GiB free under {tempfile.gettempdir()} (set TMPDIR or --mds-samples)")
    root = ddist.broadcast_object(tempfile.mkdtemp(prefix="dbx_bench_mds_") if info.rank == 0 else None)
    part = os.path.join(root, f"part{info.rank}")
    rng = np.random.default_rng(100 + info.rank)
    t0 = time.time()
    with MDSWriter(part, {"image": "pil", "label": "int"}, compression="zstd", size_limit=1 << 26) as w:
        for _ in range(n):
            w.write({"image": Image.fromarray(rng.integers(0, 256, (s, s, 3), dtype=np.uint8)),
                     "label": int(rng.integers(0, args.num_classes))})
    t_write = time.time() - t0
    ddist.barrier()
    if info.rank == 0:
        shards = []
        for r in range(info.world_size):
            with open(os.path.join(root, f"part{r}", "index.json")) as f:
                for sh in json.load(f)["shards"]:
                    for k in ("raw_data", "zip_data"):
                        if sh.get(k):
                            sh[k]["basename"] = f"part{r}/" + sh[k]["basename"]
                    shards.append(sh)
        with open(os.path.join(root, "index.json"), "w") as f:
            json.dump({"version": 2, "shards": shards}, f)
        StreamingDataset(local=root)  # decompress every shard once, before the other ranks open it
        atexit.register(shutil.rmtree, root, True)
    ddist.barrier()
    ds = StreamingDataset(local=root, shuffle=True, batch_size=B)
    aug = AugmentSpec(mode="random_crop", pad=4 if s == 32 else 0, hflip=True)
    ld = NativeImageLoader(ds, B, (s, s), tr.dev, augment=aug, nthreads=8, prefetch=3)
    state = {"it": iter(ld), "epoch": 0}

    def next_batch():
        try:
            return next(state["it"])
        except StopIteration:
            state["epoch"] += 1
            ld.set_epoch(state["epoch"])
            state["it"] = iter(ld)
            return next(state["it"])

    def step():
        img, lab, boxes, flips = next_batch()
        tr.step(img, lab, boxes, flips)

    desc = (f"{n} samples per rank in {len(ds.shards)} shards (written in {t_write:.1f} s), C++ reader "
            f"{'on' if ld.native is not None else 'off'}, pinned ring + copy stream")
    return step, desc
