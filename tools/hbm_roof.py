#!/usr/bin/env python3
"""Achievable HBM bandwidth on this GPU with stock PyTorch-ROCm kernels: read + write (copy), read
only (sum), write only (fill), over buffers well past the 256 MB last-level cache. The per-op roof
the HBM-bound convolutions are judged against (tools/op_breakdown.py reports TB/s of minimum bytes).

  python tools/hbm_roof.py [--gib 2] [--iters 20]
"""
import argparse

import torch


def bench(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=2.0)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    n = int(a.gib * (1 << 30)) // 2
    x = torch.randn(n, device="cuda", dtype=torch.bfloat16)
    y = torch.empty_like(x)
    b = 2 * n
    rows = [("copy (read + write)", lambda: y.copy_(x), 2 * b),
            ("sum (read)", lambda: torch.sum(x, dtype=torch.float32), b),
            ("fill (write)", lambda: y.fill_(1.0), b),
            ("add x + y -> y (2 reads + write)", lambda: y.add_(x), 3 * b)]
    for name, fn, nbytes in rows:
        t = bench(fn, a.iters)
        print(f"{name:34s} {nbytes / t / 1e12:6.2f} TB/s  ({t * 1e3:.3f} ms for {nbytes / 2**30:.1f} GiB)")


if __name__ == "__main__":
    main()
