#!/usr/bin/env python3
"""1x1 stride-1 weight gradients -- dW[OC, IC] = dY[P, OC]^T X[P, IC], a plain GEMM over the pixels --
on the native split-K kernel (K.conv_wgrad, tune-table tile) vs hipBLASLt through torch.mm(...,
out_dtype=float32), at the ResNet-50 b1024 shapes; plus run-to-run determinism of each."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dbx_distributed_pytorch_examples_amd.ops import kernels as K  # noqa: E402

SHAPES = [  # (H, IC, OC) of the 1x1 stride-1 convs at batch N
    (56, 64, 64), (56, 256, 64), (56, 64, 256), (56, 256, 128),
    (28, 512, 128), (28, 128, 512), (28, 512, 256),
    (14, 1024, 256), (14, 256, 1024), (14, 1024, 512),
    (7, 2048, 512), (7, 512, 2048),
]


def timeit(f, n=20):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        f()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


def main():
    N = int(os.environ.get("BATCH", 1024))
    dev = torch.device("cuda")
    ws = torch.empty(64 << 20, device=dev)
    tot_n = tot_b = 0.0
    for H, IC, OC in SHAPES:
        dy = torch.randn(N, H, H, OC, device=dev).bfloat16()
        x = torch.randn(N, H, H, IC, device=dev).bfloat16()
        dw = torch.empty(OC, IC, device=dev)
        P = N * H * H
        fn = lambda: K.conv_wgrad(dy, x, dw, ws, R=1, S=1, stride=1, pad=0)  # noqa: E731
        a2, b2 = dy.view(P, OC), x.view(P, IC)
        fb = lambda: torch.mm(a2.t(), b2, out_dtype=torch.float32)  # noqa: E731
        tn, tb = timeit(fn), timeit(fb)
        fn()
        r1 = dw.clone()
        fn()
        det_n = torch.equal(r1, dw)
        o1, o2 = fb(), fb()
        det_b = torch.equal(o1, o2)
        err = ((o1 - r1).abs().max() / r1.abs().max()).item()
        fl = 2.0 * P * OC * IC
        tot_n += tn
        tot_b += tb
        print(f"{IC:5d}->{OC:5d} @{H:3d}: native {tn*1e3:7.1f} us ({fl/tn/1e9:6.0f} TF/s, det {det_n}) | "
              f"hipBLASLt {tb*1e3:7.1f} us ({fl/tb/1e9:6.0f} TF/s, det {det_b}) | rel diff {err:.2e}", flush=True)
    print(f"total: native {tot_n*1e3:.0f} us, hipBLASLt {tot_b*1e3:.0f} us")


if __name__ == "__main__":
    main()
