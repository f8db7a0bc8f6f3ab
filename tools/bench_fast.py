#!/usr/bin/env python3
"""A/B of the eight-wave conv kernel (csrc/conv_fast.hip, tile (256, bn, 4)) against the four-wave
implicit-GEMM tiles on the compute-bound ResNet-50 b1024 conv shapes with plain operands.

For each shape: checks the fast kernel's output (and BN statistics) bit-for-bit against the
reference tile (same K order -> identical fp32 sums), then times interleaved rounds in one process
(cdna_hip_programming.md §5.4 rule 24) and prints median ms and TF/s per variant.
  python tools/bench_fast.py [--batch 1024] [--rounds 5] [--iters 10]
"""
import argparse
import json
import math
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dbx_distributed_pytorch_examples_amd.ops import kernels as K  # noqa: E402

# (name, mode, C_in, C_out, R, H, epi, variants)
# variant tuples: (bm, bn, dma) -- dma 4 = the eight-wave kernel with the full-rounds batch split;
# (256, bn, 4, 0) = the eight-wave kernel over the whole batch (partial last round)
CASES = [
    ("dgrad3x3@14 256 epi2", "dgrad", 256, 256, 3, 14, 2, [(128, 128, 2), (256, 128, 4, 0), (256, 128, 4)]),
    ("dgrad3x3@28 128 epi2", "dgrad", 128, 128, 3, 28, 2, [(128, 128, 2), (256, 128, 4)]),
    ("dgrad3x3@7 512 epi2", "dgrad", 512, 512, 3, 7, 2, [(128, 128, 2), (256, 128, 4)]),
    ("fwd3x3@14 256 stats", "fwd", 256, 256, 3, 14, 0, [(128, 256, 0), (256, 256, 4, 0), (256, 256, 4)]),
    ("fwd3x3@28 128 stats", "fwd", 128, 128, 3, 28, 0, [(128, 128, 0), (256, 128, 4, 0), (256, 128, 4)]),
    ("fwd3x3@7 512 stats", "fwd", 512, 512, 3, 7, 0, [(128, 256, 0), (256, 256, 4, 0), (256, 256, 4)]),
    ("fwd1x1@14 256->1024 stats", "fwd", 256, 1024, 1, 14, 0, [(128, 256, 0), (256, 256, 4, 0), (256, 256, 4)]),
    ("fwd1x1@28 128->512 stats", "fwd", 128, 512, 1, 28, 0, [(128, 256, 0), (256, 256, 4, 0), (256, 256, 4)]),
    ("fwd1x1@7 512->2048 stats", "fwd", 512, 2048, 1, 7, 0, [(128, 256, 0), (256, 256, 4, 0), (256, 256, 4)]),
    ("dgrad1x1@14 1024->256 epi2", "dgrad", 256, 1024, 1, 14, 2, [(128, 128, 2), (256, 128, 4)]),
    ("dgrad1x1@14 256->1024 epi1", "dgrad", 1024, 256, 1, 14, 1, [(128, 128, 2), (256, 256, 4, 0), (256, 256, 4)]),
    ("dgrad1x1@7 512->2048 epi1", "dgrad", 2048, 512, 1, 7, 1, [(128, 128, 2), (256, 256, 4, 0), (256, 256, 4)]),
    ("dgrad3x3@14 256 epi0", "dgrad", 256, 256, 3, 14, 0, [(128, 128, 2), (256, 256, 4, 0), (256, 256, 4)]),
]


def timeit(fn, iters):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def build(case, N, dev):
    name, mode, C, Kc, R, H, epi, variants = case
    pad = R // 2
    torch.manual_seed(0)
    if mode == "fwd":
        x = torch.randn(N, H, H, C, device=dev).bfloat16()
        w = (torch.randn(Kc, R * R * C, device=dev) / math.sqrt(C * R * R)).bfloat16()
        outs = {}

        def make(tile):
            y = torch.empty(N, H, H, Kc, device=dev, dtype=torch.bfloat16)
            st = K.new_stats(Kc, dev)

            def run():
                st.zero_()
                K.conv_fwd(x, w, y, R=R, S=R, stride=1, pad=pad, stats=st, tile=tile[:3], _split=tile[3:4] != (0,))
            outs[tile] = (y, st)
            return run
        flops = 2.0 * N * H * H * Kc * R * R * C
        return make, outs, flops
    # dgrad: dy [N,H,H,Kc(=out of fwd)] -> dx [N,H,H,C]; here "C" = dx channels, "Kc" = dy channels
    dy = torch.randn(N, H, H, Kc, device=dev).bfloat16()
    wt = (torch.randn(C, R * R * Kc, device=dev) / math.sqrt(Kc * R * R)).bfloat16()
    ybn = torch.randn(N, H, H, C, device=dev).bfloat16()
    mean, inv = torch.randn(C, device=dev) * 0.1, torch.rand(C, device=dev) + 0.5
    sc, sh = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1
    mb = K.pack_mask_bits(torch.randn(N, H, H, C, device=dev))
    outs = {}

    def make(tile):
        dx = torch.empty(N, H, H, C, device=dev, dtype=torch.bfloat16)
        st = K.new_stats(C, dev)
        act = torch.empty_like(dx) if epi == 2 else None
        if epi == 2:
            e = K.BNBwdEpilogue(K.MASK_Y, ybn, mean, inv, st, scale=sc, shift=sh, act_out=act)
        elif epi == 1:
            e = K.BNBwdEpilogue(K.MASK_OUT, ybn, mean, inv, st, mbits=mb)
        else:
            e = None

        def run():
            st.zero_()
            K.conv_dgrad(dy, wt, dx, R=R, S=R, stride=1, pad=pad, tile=tile[:3], epilogue=e,
                         _split=tile[3:4] != (0,))
        outs[tile] = (dx, st)
        return run
    flops = 2.0 * N * H * H * Kc * R * R * C
    return make, outs, flops


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    dev = torch.device("cuda")
    results = []
    for case in CASES:
        if a.only and a.only not in case[0]:
            continue
        make, outs, flops = build(case, a.batch, dev)
        variants = list(case[7])
        runs = {t: make(t) for t in variants}
        for r in runs.values():
            r()
        torch.cuda.synchronize()
        ref_t = variants[0]
        ok = {}
        for t in variants[1:]:
            y0, s0 = outs[ref_t]
            y1, s1 = outs[t]
            same = torch.equal(y0, y1)
            rel = ((y1.float() - y0.float()).norm() / y0.float().norm()).item()
            # statistics shards differ with the tile geometry: compare the shard sums
            a0, a1 = s0.view(K.NSHARD, -1).sum(0), s1.view(K.NSHARD, -1).sum(0)
            srel = ((a1 - a0).norm() / a0.norm().clamp_min(1e-30)).item()
            ok[str(t)] = {"bit_equal": same, "rel": rel, "stats_rel": srel}
        times = {t: [] for t in runs}
        for _ in range(a.rounds):
            for t, r in runs.items():
                times[t].append(timeit(r, a.iters))
        row = {"case": case[0], "check": ok}
        for t in runs:
            ms = statistics.median(times[t])
            row[str(t)] = {"ms": round(ms, 4), "tf": round(flops / ms / 1e9, 1)}
        results.append(row)
        print(json.dumps(row), flush=True)
        del runs, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
