#!/usr/bin/env python3
"""Cost of the forward BN-statistics epilogue: the 1x1 expansion convs (C -> 4C) and the 3x3 convs
of ResNet-50 b1024 with and without ``stats=`` (same tile from the tune table), BN prologue on."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dbx_distributed_pytorch_examples_amd.ops import kernels as k  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


N, dev = 1024, "cuda"
for (H, C, Kc, R) in ((56, 64, 256, 1), (28, 128, 512, 1), (14, 256, 1024, 1), (7, 512, 2048, 1),
                      (28, 128, 128, 3), (14, 256, 256, 3), (7, 512, 512, 3)):
    x = torch.randn(N, H, H, C, device=dev).bfloat16()
    w = (torch.randn(Kc, R * R * C, device=dev) / (C * R * R) ** 0.5).bfloat16()
    y = torch.empty(N, H, H, Kc, device=dev, dtype=torch.bfloat16)
    st = k.new_stats(Kc, dev)
    sc, sh = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1
    t_st = timeit(lambda: k.conv_fwd(x, w, y, R=R, S=R, stride=1, pad=R // 2, stats=st, in_scale=sc, in_shift=sh))
    t_no = timeit(lambda: k.conv_fwd(x, w, y, R=R, S=R, stride=1, pad=R // 2, in_scale=sc, in_shift=sh))
    print(f"{H}x{H} {C}->{Kc} {R}x{R}: with stats {t_st:.3f} ms, without {t_no:.3f} ms "
          f"(stats epilogue {100 * (t_st - t_no) / t_st:.1f} %)", flush=True)
