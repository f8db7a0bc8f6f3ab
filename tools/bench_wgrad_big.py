#!/usr/bin/env python3
"""Weight-gradient microbenchmark: the tune table's choice vs the 256 x 256 tile (dma 4: 32-pixel
stages in a 4-slot ring; dma 2: 64-pixel stages in 2 slots) at several split depths, for every
ResNet-50 @224 weight gradient whose OC and IC are multiples of 256. Interleaved rounds, medians,
random data (cdna_hip_programming.md §5.4 rules 24 / 25).
  python tools/bench_wgrad_big.py --batch 1024
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dbx_distributed_pytorch_examples_amd.ops import kernels as K  # noqa: E402

R50 = [  # C, K, R, stride, H_in (ResNet-50 @224 convs)
    (64, 64, 1, 1, 56), (64, 64, 3, 1, 56), (64, 256, 1, 1, 56), (256, 64, 1, 1, 56), (256, 128, 1, 1, 56),
    (128, 128, 3, 2, 56), (128, 512, 1, 1, 28), (256, 512, 1, 2, 56), (512, 128, 1, 1, 28), (128, 128, 3, 1, 28),
    (512, 256, 1, 1, 28), (256, 256, 3, 2, 28), (256, 1024, 1, 1, 14), (512, 1024, 1, 2, 28),
    (1024, 256, 1, 1, 14), (256, 256, 3, 1, 14), (1024, 512, 1, 1, 14), (512, 512, 3, 2, 14),
    (512, 2048, 1, 1, 7), (1024, 2048, 1, 2, 14), (2048, 512, 1, 1, 7), (512, 512, 3, 1, 7),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--splits", default="0.5,1,2")
    a = ap.parse_args()
    N, dev = a.batch, "cuda"
    ws = torch.empty(512 * 1024 * 1024 // 4, device=dev)
    total = {"table": 0.0, "best": 0.0}
    for (C, Kc, R, st, H) in R50:
        if C % 256 or Kc % 256:
            continue
        pad = R // 2
        OH = (H + 2 * pad - R) // st + 1
        x = torch.randn(N, H, H, C, device=dev).bfloat16()
        dy = torch.randn(N, OH, OH, Kc, device=dev).bfloat16()
        dw = torch.empty(Kc, R * R * C, device=dev)
        cnt = torch.zeros(K.wgrad_tiles_max(Kc, R * R * C), dtype=torch.int32, device=dev)
        ref = torch.empty_like(dw)
        K.conv_wgrad(dy, x, ref, ws, R=R, S=R, stride=st, pad=pad, cnt=cnt)
        cands = {"table": dict()}
        for d in (4, 2):
            for r in a.splits.split(","):
                cands[f"256x256 dma{d} r{r}"] = dict(tile=(256, 256), dma=d, rounds=float(r))
        times = {k: [] for k in cands}
        flop = 2.0 * N * OH * OH * Kc * R * R * C
        for _ in range(a.rounds):
            for name, kw in cands.items():
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    K.conv_wgrad(dy, x, dw, ws, R=R, S=R, stride=st, pad=pad, cnt=cnt, **kw)
                e1.record()
                torch.cuda.synchronize()
                times[name].append(e0.elapsed_time(e1) / a.iters)
        err = ((dw - ref).norm() / ref.norm()).item()
        med = {k: statistics.median(v) for k, v in times.items()}
        best = min(med, key=med.get)
        total["table"] += med["table"]
        total["best"] += med[best]
        line = " | ".join(f"{k} {v * 1e3:.0f}us ({flop / v / 1e9:.0f}TF)" for k, v in med.items())
        print(f"wgrad {C}->{Kc} {R}x{R} s{st} @{OH}: {line} | best {best} (rel err last {err:.1e})", flush=True)
        del x, dy, dw
    print(f"sum over shapes (one call each): table {total['table']:.3f} ms, best {total['best']:.3f} ms")


if __name__ == "__main__":
    main()
