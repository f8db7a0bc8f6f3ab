#!/usr/bin/env python3
"""Library ceiling check: hipBLASLt (torch.mm, bf16) on the plain-GEMM shapes of ResNet-50's 1x1
convs at batch 1024 (NHWC: [pixels, C_in] x [C_in, C_out]) vs the dbx conv kernel without fusions."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dbx_distributed_pytorch_examples_amd.ops import kernels as K  # noqa: E402


def t(fn, it=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


N = 1024
for C, Kc, H in [(64, 256, 56), (256, 64, 56), (128, 512, 28), (512, 128, 28), (256, 1024, 14), (1024, 256, 14),
                 (512, 2048, 7), (2048, 512, 7)]:
    M = N * H * H
    a = torch.randn(M, C, device="cuda").bfloat16()
    b = torch.randn(C, Kc, device="cuda").bfloat16()
    bt = b.t().contiguous()
    o = torch.empty(M, Kc, device="cuda", dtype=torch.bfloat16)
    ms_lib = t(lambda: torch.mm(a, b, out=o))
    ms_dbx = t(lambda: K.conv_fwd(a.view(N, H, H, C), bt, o.view(N, H, H, Kc), R=1, S=1, stride=1, pad=0))
    fl = 2.0 * M * C * Kc
    by = (M * C + M * Kc) * 2
    print(f"{C:5d}->{Kc:5d} @{H:3d}: hipBLASLt {ms_lib:.3f} ms ({fl / ms_lib / 1e9:.0f} TF/s, {by / ms_lib / 1e9:.2f} TB/s)"
          f" | dbx {ms_dbx:.3f} ms ({fl / ms_dbx / 1e9:.0f} TF/s, {by / ms_dbx / 1e9:.2f} TB/s)", flush=True)
