#!/usr/bin/env python3
"""Input-pipeline throughput (SURVEY.md §7.2 step 5 gate: loader >= 2x the model's img/s per rank):
writes an MDS dataset of raw uint8 images (TinyImageNet-shaped by default), then times
``data.loader.NativeImageLoader`` over it: C++ shard reader (mmap + thread pool) -> pinned staging
ring -> async H2D copy on the copy stream (+ host-sampled crop boxes / flips for the GPU augment).

  python tools/bench_loader.py [--n 20000] [--size 64] [--batch 512] [--threads 8] [--device cuda]
"""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dbx_distributed_pytorch_examples_amd.data.loader import AugmentSpec, NativeImageLoader  # noqa: E402
from dbx_distributed_pytorch_examples_amd.data.mds import MDSWriter, StreamingDataset  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=20000)
    ap.add_argument("--size", type=int, default=64)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--epochs", type=int, default=2)
    ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    a = ap.parse_args()
    tmp = tempfile.mkdtemp(prefix="dbx_mds_")
    try:
        rng = np.random.default_rng(0)
        t0 = time.time()
        with MDSWriter(tmp, {"image": f"ndarray:uint8:{a.size},{a.size},3", "label": "int"}, size_limit=1 << 26) as w:
            for i in range(a.n):
                w.write({"image": rng.integers(0, 256, (a.size, a.size, 3), dtype=np.uint8), "label": i % 200})
        t_write = time.time() - t0
        ds = StreamingDataset(local=tmp, shuffle=True, batch_size=a.batch)
        dev = torch.device(a.device)
        ld = NativeImageLoader(ds, a.batch, (a.size, a.size), dev, nthreads=a.threads, prefetch=2,
                               augment=AugmentSpec(mode="random_crop", pad=4, hflip=True))
        res = []
        for ep in range(a.epochs):
            ld.set_epoch(ep)
            n = 0
            t0 = time.time()
            for img, lab, boxes, flips in ld:
                n += img.shape[0]
            if dev.type == "cuda":
                torch.cuda.synchronize()
            dt = time.time() - t0
            res.append(round(n / dt, 1))
        out = {"images_per_s": res, "native_reader": ld.native is not None, "device": a.device,
               "batch": a.batch, "image": [a.size, a.size, 3], "threads": a.threads,
               "mds_write_s": round(t_write, 2), "samples": a.n}
        print(json.dumps(out))
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
