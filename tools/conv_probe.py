#!/usr/bin/env python3
"""Run single conv kernels of the ResNet-50 b1024 step in isolation (for rocprofv3 --pmc passes).

  python tools/conv_probe.py --case fwd3x3_64 --tile 128,64,1 --iters 5

Cases (C->K, geometry @ input size, batch 1024):
  fwd3x3_64   64->64 3x3 s1 @56, BN prologue + stats epilogue (the bottleneck conv2 forward)
  dgrad3x3_64 its data gradient with the MASK_Y BN-backward epilogue (+ BN-output write-back)
  fwd3x3_128  / dgrad3x3_128   the same at 128 channels @28
  fwd3x3_256  / dgrad3x3_256   the same at 256 channels @14
Prints the median time per launch.
"""
import argparse
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dbx_distributed_pytorch_examples_amd.ops import kernels as K  # noqa: E402

GEOM = {"64": (64, 56), "128": (128, 28), "256": (256, 14), "512": (512, 7)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="fwd3x3_64")
    ap.add_argument("--tile", default="")
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    kind, ch = a.case.split("3x3_")
    C, H = GEOM[ch]
    N, dev = a.batch, "cuda"
    tile = (a.tile if a.tile.startswith("patch") else tuple(int(v) for v in a.tile.split(","))) if a.tile else None
    torch.manual_seed(0)
    x = torch.randn(N, H, H, C, device=dev).bfloat16()
    w = (torch.randn(C, 9 * C, device=dev) / math.sqrt(9 * C)).bfloat16()
    sc, sh = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1
    y = torch.empty_like(x)
    st = K.new_stats(C, dev)
    if kind == "fwd":
        def run():
            K.conv_fwd(x, w, y, R=3, S=3, stride=1, pad=1, stats=st, in_scale=sc, in_shift=sh, tile=tile)
    else:
        wt = w.view(C, 3, 3, C).permute(3, 1, 2, 0).contiguous().view(C, -1)
        ybn, act = torch.randn_like(x), torch.empty_like(x)
        mean, inv = torch.randn(C, device=dev) * 0.1, torch.rand(C, device=dev) + 0.5
        e = K.BNBwdEpilogue(K.MASK_Y, ybn, mean, inv, st, scale=sc, shift=sh, act_out=act)

        def run():
            K.conv_dgrad(x, wt, y, R=3, S=3, stride=1, pad=1, epilogue=e, tile=tile)
    run()
    torch.cuda.synchronize()
    ts = []
    for _ in range(a.iters):
        s, e2 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        run()
        e2.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e2))
    ms = sorted(ts)[len(ts) // 2]
    fl = 2.0 * N * H * H * C * 9 * C
    print(f"{a.case} tile={tile} {ms:.3f} ms  {fl / ms / 1e9:.0f} TF/s")


if __name__ == "__main__":
    main()
