#!/usr/bin/env python3
"""Cost breakdown of the memory-bound convs: fwd plain / +prologue / +stats, dgrad plain / +epilogues,
against a same-bytes copy (the achievable HBM roof). Prints effective TB/s per variant."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dbx_distributed_pytorch_examples_amd.ops import kernels as K  # noqa: E402


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    dev = "cuda"
    N = int(os.environ.get("BATCH", 1024))
    shapes = [(64, 256, 56), (256, 64, 56), (256, 128, 56), (512, 128, 28), (1024, 256, 14), (256, 1024, 14)]
    tiles = [None, (128, 128), (128, 256), (256, 128), (256, 64), (128, 64)]
    big = torch.empty(2 * 1024 ** 3 // 2, device=dev, dtype=torch.bfloat16)
    big2 = torch.empty_like(big)
    t = timeit(lambda: big2.copy_(big))
    print(f"copy 2 GiB: {t:.3f} ms  {2 * 2 * 2 ** 30 / t / 1e9:.2f} TB/s (read+write)")
    if os.environ.get("ONLY_WGRAD"):
        tiles = []
    for C, Kc, H in shapes:
        x = torch.randn(N, H, H, C, device=dev).bfloat16()
        w = (torch.randn(Kc, C, device=dev) / math.sqrt(C)).bfloat16()
        y = torch.empty(N, H, H, Kc, device=dev, dtype=torch.bfloat16)
        stats = K.new_stats(Kc, dev)
        sc, sh = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1
        byt = (x.numel() + y.numel()) * 2
        print(f"--- {C}->{Kc} @{H}  fwd bytes {byt / 1e9:.2f} GB, copy-roof {byt / 6.0e9:.3f} ms")
        for tile in tiles:
            if tile and Kc % tile[1]:
                continue
            r = []
            for pro, st in ((0, 0), (1, 0), (0, 1), (1, 1)):
                f = lambda: K.conv_fwd(x, w, y, R=1, S=1, stride=1, pad=0, stats=stats if st else None,  # noqa: E731
                                       in_scale=sc if pro and C <= 512 else None,
                                       in_shift=sh if pro and C <= 512 else None, tile=tile)
                ms = timeit(f)
                r.append(f"{'P' if pro else '-'}{'S' if st else '-'} {ms:.3f}ms/{byt / ms / 1e9:.1f}TB/s")
            print(f"  fwd tile {tile}: " + "  ".join(r))
        # dgrad of the same conv: dy [N,H,H,Kc] -> dx [N,H,H,C]
        dy = torch.randn(N, H, H, Kc, device=dev).bfloat16()
        wt = w.t().contiguous()
        dx = torch.empty_like(x)
        ybn, mref, add = torch.randn_like(x), torch.randn_like(x), torch.randn_like(x)
        st1 = K.new_stats(C, dev)
        mean, inv = torch.randn(C, device=dev) * 0.1, torch.rand(C, device=dev) + 0.5
        e1 = K.BNBwdEpilogue(K.MASK_OUT, ybn, mean, inv, st1, mbits=K.pack_mask_bits(mref))
        e2 = K.BNBwdEpilogue(K.MASK_Y, ybn, mean, inv, st1, scale=sc, shift=sh)
        for tile in tiles:
            if tile and C % tile[1]:
                continue
            r = []
            for name, kw, nb in (("plain", {}, 2), ("acc", dict(addsrc=add), 3), ("e2", dict(epilogue=e2), 3),
                                 ("e1+acc", dict(epilogue=e1, addsrc=add), 5)):
                ms = timeit(lambda: K.conv_dgrad(dy, wt, dx, R=1, S=1, stride=1, pad=0, tile=tile, **kw))
                b2 = dy.numel() * 2 + nb * dx.numel() * 2
                r.append(f"{name} {ms:.3f}ms/{b2 / ms / 1e9:.1f}TB/s")
            print(f"  dgrad tile {tile}: " + "  ".join(r))
        ws = torch.empty(max(64 * Kc * C, 16 << 20), device=dev)
        dw = torch.empty(Kc * C, device=dev)
        r = []
        for pro in (0, 1):
            ms = timeit(lambda: K.conv_wgrad(dy, x, dw, ws, R=1, S=1, stride=1, pad=0, in_scale=sc if pro else None,
                                             in_shift=sh if pro else None))
            r.append(f"{'P' if pro else '-'} {ms:.3f}ms/{2 * N * H * H * Kc * C / ms / 1e9:.0f}TF/s")
        print("  wgrad: " + "  ".join(r))
        del x, y, dy, dx, ybn, mref, add
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
