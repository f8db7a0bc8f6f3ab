#!/usr/bin/env python3
"""Per-tile cost of the 1x1 short-K convs (the N-sweep question): how does the time of a
BN-prologue forward / folded-TAIL data gradient split between the K loop (A staging + prologue,
B, MFMA) and the epilogue? Times the implicit-GEMM kernel at a fixed tile over K (input channels
of the GEMM) and N (output channels), M = batch x H x W.

  python tools/probe_sweep.py [--batch 1024] [--iters 10]
"""
import argparse
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dbx_distributed_pytorch_examples_amd.ops import kernels as K  # noqa: E402


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def fwd_case(N, H, IC, OC, tile, iters):
    dev = "cuda"
    x = torch.randn(N, H, H, IC, device=dev).bfloat16()
    w = (torch.randn(OC, IC, device=dev) / math.sqrt(IC)).bfloat16()
    y = torch.empty(N, H, H, OC, device=dev, dtype=torch.bfloat16)
    sc, sh = torch.rand(IC, device=dev) + 0.5, torch.randn(IC, device=dev) * 0.1
    st = K.new_stats(OC, dev)
    return timeit(lambda: K.conv_fwd(x, w, y, R=1, S=1, stride=1, pad=0, stats=st, in_scale=sc, in_shift=sh,
                                     tile=tile), iters)


def dgrad_case(N, H, Kc, Cc, tile, iters):
    """conv1 data gradient of a bottleneck (Cc -> Kc conv): the BN1-backward apply folded into the
    operand staging, the block-input addend and the previous block's MASK_OUT epilogue."""
    dev = "cuda"
    g = torch.randn(N, H, H, Kc, device=dev).bfloat16()
    yb = torch.randn(N, H, H, Kc, device=dev).bfloat16()
    coeff = torch.randn(3, Kc, device=dev) * 0.1
    dyo = torch.empty_like(g)
    wt = (torch.randn(Cc, Kc, device=dev) / math.sqrt(Kc)).bfloat16()
    dx = torch.empty(N, H, H, Cc, device=dev, dtype=torch.bfloat16)
    add = torch.randn_like(dx)
    ybn = torch.randn_like(dx)
    mb = K.pack_mask_bits(torch.randn(N, H, H, Cc, device=dev) > 0)
    m1, i1 = torch.randn(Cc, device=dev) * 0.1, torch.rand(Cc, device=dev) + 0.5
    st = K.new_stats(Cc, dev)
    epi = K.BNBwdEpilogue(K.MASK_OUT, ybn, m1, i1, st, mbits=mb)
    return timeit(lambda: K.conv_dgrad(g, wt, dx, R=1, S=1, stride=1, pad=0, tile=tile, addsrc=add, epilogue=epi,
                                       bwd_y=yb, bwd_coeff=coeff, dy_out=dyo), iters)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--sweep", action="store_true", help="the N-sweep forward (tile dma 8) against the 128 x 256 igemm tile")
    a = ap.parse_args()
    N = a.batch
    if a.sweep:
        print(f"# batch {N}: 1x1 BN-prologue forwards + stats, igemm 128x256 vs N-sweep (us per launch)", flush=True)
        for H, IC, OC in ((28, 128, 512), (14, 256, 1024), (56, 64, 256), (28, 64, 512), (14, 128, 1024)):
            t0 = min(fwd_case(N, H, IC, OC, (128, 256, 1), a.iters) for _ in range(3))
            t1 = min(fwd_case(N, H, IC, OC, (128, 256, 8), a.iters) for _ in range(3))
            by = N * H * H * (IC + OC) * 2
            print(f"fwd {IC:4d}->{OC:5d} @{H:2d}: igemm {t0 * 1e3:7.1f} us ({by / t0 / 1e9:4.2f} TB/s)  "
                  f"sweep {t1 * 1e3:7.1f} us ({by / t1 / 1e9:4.2f} TB/s)  {t0 / t1:5.2f}x", flush=True)
        print("# folded conv1 data gradients + addend + MASK_OUT epilogue", flush=True)
        for H, Kc, Cc in ((14, 256, 1024), (28, 128, 512), (56, 64, 256)):
            t0 = min(dgrad_case(N, H, Kc, Cc, (128, 256, 1), a.iters) for _ in range(3))
            t1 = min(dgrad_case(N, H, Kc, Cc, (128, 256, 8), a.iters) for _ in range(3))
            by = N * H * H * (3 * Kc + 3 * Cc) * 2
            print(f"dgrad {Kc:4d}->{Cc:5d} @{H:2d}: igemm {t0 * 1e3:7.1f} us ({by / t0 / 1e9:4.2f} TB/s)  "
                  f"sweep {t1 * 1e3:7.1f} us ({by / t1 / 1e9:4.2f} TB/s)  {t0 / t1:5.2f}x", flush=True)
        return
    tile = (128, 256, 1)
    print(f"# batch {N}, tile {tile}: per-tile us = time / (M/128 * N/256)", flush=True)
    for kind, fn in (("fwd pro+stats", fwd_case), ("dgrad fold epi1", dgrad_case)):
        for H, ks, ns in ((14, (64, 128, 256), (256, 512, 1024)), (28, (64, 128), (256, 512))):
            for kk in ks:
                for nn in ns:
                    t = min(fn(N, H, kk, nn, tile, a.iters) for _ in range(3))
                    ntile = (N * H * H // 128) * (nn // 256)
                    print(f"{kind:16s} @{H:2d} K {kk:4d} N {nn:5d}: {t * 1e3:8.1f} us  per tile-CU "
                          f"{t * 1e3 * 256 / ntile:6.2f} us", flush=True)


if __name__ == "__main__":
    main()
