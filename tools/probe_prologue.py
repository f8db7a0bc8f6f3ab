#!/usr/bin/env python3
"""Is the BN prologue worth re-doing per N tile? For the bottleneck conv3 forwards (1x1, C -> 4C) time
(a) conv with the BN-apply+ReLU prologue + stats epilogue (the program's schedule) against
(b) a bn_apply pass materialising relu(bn(x)) + the prologue-free conv (+ stats), at ResNet-50 b1024."""
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
for (H, C) in ((56, 64), (28, 128), (14, 256), (7, 512)):
    Kc = 4 * C
    x = torch.randn(N, H, H, C, device=dev).bfloat16()
    w = (torch.randn(Kc, C, device=dev) / C ** 0.5).bfloat16()
    y = torch.empty(N, H, H, Kc, device=dev, dtype=torch.bfloat16)
    a = torch.empty_like(x)
    st = k.new_stats(Kc, dev)
    sc, sh = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1
    t_pro = timeit(lambda: k.conv_fwd(x, w, y, R=1, S=1, stride=1, pad=0, stats=st, in_scale=sc, in_shift=sh))
    t_app = timeit(lambda: k.bn_apply(x, sc, sh, a, relu=True))
    res = []
    for tile in (None, (128, 256, 2), (128, 256, 3), (128, 128, 2), (256, 128, 2), (128, 256, 0)):
        try:
            t = timeit(lambda: k.conv_fwd(a, w, y, R=1, S=1, stride=1, pad=0, stats=st, tile=tile))
            res.append(f"{tile}: {t:.3f}")
        except Exception as e:  # noqa: BLE001
            res.append(f"{tile}: n/a ({str(e)[:40]})")
    print(f"{H}x{H} {C}->{Kc}: prologue conv {t_pro:.3f} ms | bn_apply {t_app:.3f} + plain conv " + ", ".join(res),
          flush=True)
