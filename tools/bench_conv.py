#!/usr/bin/env python3
"""Per-shape conv microbenchmark: dbx HIP implicit-GEMM vs MIOpen (torch channels_last bf16).

Shapes = the unique ResNet-50 @224 convs of SURVEY.md §2.4. Times are medians of interleaved
rounds in one process (cdna_hip_programming.md §5.4 rule 24), random data.
  python tools/bench_conv.py --batch 256 [--out profiles/conv_bench.md]
"""
import argparse
import math
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dbx_distributed_pytorch_examples_amd.ops import kernels as K  # noqa: E402

R50 = [  # C, K, R, stride, H_in
    (64, 64, 1, 1, 56), (64, 64, 3, 1, 56), (64, 256, 1, 1, 56), (256, 64, 1, 1, 56), (256, 128, 1, 1, 56),
    (128, 128, 3, 2, 56), (128, 512, 1, 1, 28), (256, 512, 1, 2, 56), (512, 128, 1, 1, 28), (128, 128, 3, 1, 28),
    (512, 256, 1, 1, 28), (256, 256, 3, 2, 28), (256, 1024, 1, 1, 14), (512, 1024, 1, 2, 28),
    (1024, 256, 1, 1, 14), (256, 256, 3, 1, 14), (1024, 512, 1, 1, 14), (512, 512, 3, 2, 14),
    (512, 2048, 1, 1, 7), (1024, 2048, 1, 2, 14), (2048, 512, 1, 1, 7), (512, 512, 3, 1, 7),
]


def timeit(fn, iters=10):
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(iters):
        fn()
    ev1.record()
    torch.cuda.synchronize()
    return ev0.elapsed_time(ev1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    N = a.batch
    dev = "cuda"
    ws = torch.empty(256 * 1024 * 1024 // 4 * 4, device=dev)
    lines = ["| C→K | R s | H | GFLOP | dbx fwd ms (TF) | miopen fwd ms | dbx dgrad ms | miopen dgrad ms | dbx wgrad ms | miopen wgrad ms |",
             "|---|---|---|---|---|---|---|---|---|---|"]
    tot = {"dbx": [0, 0, 0], "mio": [0, 0, 0]}
    for (C, Kc, R, st, H) in R50:
        pad = R // 2
        OH = (H + 2 * pad - R) // st + 1
        x = torch.randn(N, H, H, C, device=dev).bfloat16()
        w = (torch.randn(Kc, R, R, C, device=dev) / math.sqrt(C * R * R)).bfloat16()
        wt = w.permute(3, 1, 2, 0).contiguous().view(C, -1)
        w2 = w.view(Kc, -1)
        y = torch.empty(N, OH, OH, Kc, device=dev, dtype=torch.bfloat16)
        dy = torch.randn(N, OH, OH, Kc, device=dev).bfloat16()
        dx = torch.empty_like(x)
        dw = torch.empty(Kc, R * R * C, device=dev)
        stats = K.new_stats(Kc, dev)
        xc = x.permute(0, 3, 1, 2)  # channels_last view
        wc = w.permute(0, 3, 1, 2)
        dyc = dy.permute(0, 3, 1, 2)
        res = {}
        for _ in range(a.rounds):
            res.setdefault("df", []).append(timeit(lambda: K.conv_fwd(x, w2, y, R=R, S=R, stride=st, pad=pad, stats=stats)))
            res.setdefault("mf", []).append(timeit(lambda: F.conv2d(xc, wc, stride=st, padding=pad)))
            res.setdefault("dd", []).append(timeit(lambda: K.conv_dgrad(dy, wt, dx, R=R, S=R, stride=st, pad=pad)))
            res.setdefault("md", []).append(timeit(lambda: torch.ops.aten.convolution_backward(
                dyc, xc, wc, None, [st, st], [pad, pad], [1, 1], False, [0, 0], 1, [True, False, False])))
            res.setdefault("dw", []).append(timeit(lambda: K.conv_wgrad(dy, x, dw, ws, R=R, S=R, stride=st, pad=pad)))
            res.setdefault("mw", []).append(timeit(lambda: torch.ops.aten.convolution_backward(
                dyc, xc, wc, None, [st, st], [pad, pad], [1, 1], False, [0, 0], 1, [False, True, False])))
        med = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
        gf = 2.0 * N * OH * OH * Kc * C * R * R / 1e9
        for i, (d, m) in enumerate((("df", "mf"), ("dd", "md"), ("dw", "mw"))):
            tot["dbx"][i] += med[d]
            tot["mio"][i] += med[m]
        lines.append(f"| {C}→{Kc} | {R}x{R} s{st} | {H} | {gf:.1f} | {med['df']:.3f} ({gf / med['df']:.0f}) | {med['mf']:.3f} | "
                     f"{med['dd']:.3f} ({gf / med['dd']:.0f}) | {med['md']:.3f} | {med['dw']:.3f} ({gf / med['dw']:.0f}) | {med['mw']:.3f} |")
        print(lines[-1], flush=True)
    lines.append(f"| **sum (unique shapes, 1 each)** | | | | {tot['dbx'][0]:.2f} | {tot['mio'][0]:.2f} | {tot['dbx'][1]:.2f} | "
                 f"{tot['mio'][1]:.2f} | {tot['dbx'][2]:.2f} | {tot['mio'][2]:.2f} |")
    print(lines[-1])
    if a.out:
        with open(a.out, "w") as f:
            f.write(f"# conv microbenchmark, batch {N}, bf16 NHWC, MI355X\n\n" + "\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
