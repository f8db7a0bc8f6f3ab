"""Run one conv kernel shape repeatedly (for rocprofv3 counter collection).

  python tools/wgrad_one.py N C K H R {fwd|fwdps|dgrad|wgrad}
"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dbx_distributed_pytorch_examples_amd.ops import kernels as K  # noqa: E402

N, C, Kc, H, R = (int(v) for v in (sys.argv[1:6] if len(sys.argv) > 5 else (1024, 256, 256, 14, 3)))
kind = sys.argv[6] if len(sys.argv) > 6 else "wgrad"
dev = "cuda"
pad = R // 2
x = torch.randn(N, H, H, C, device=dev).bfloat16()
dy = torch.randn(N, H, H, Kc, device=dev).bfloat16()
w = (torch.randn(Kc, R, R, C, device=dev) / math.sqrt(C * R * R)).bfloat16()
ws = torch.empty(max(64 * Kc * R * R * C, 16 << 20), device=dev)
dw = torch.empty(Kc * R * R * C, device=dev)
y = torch.empty(N, H, H, Kc, device=dev, dtype=torch.bfloat16)
st = K.new_stats(Kc, dev)
sc, sh = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1
for _ in range(5):
    if kind == "wgrad":
        K.conv_wgrad(dy, x, dw, ws, R=R, S=R, stride=1, pad=pad)
    elif kind == "dgrad":
        K.conv_dgrad(dy, w.permute(3, 1, 2, 0).contiguous().view(C, -1), x, R=R, S=R, stride=1, pad=pad)
    elif kind == "fwdps":  # BN prologue + statistics epilogue (the program's forward convs)
        K.conv_fwd(x, w.view(Kc, -1), y, R=R, S=R, stride=1, pad=pad, stats=st, in_scale=sc, in_shift=sh)
    else:
        K.conv_fwd(x, w.view(Kc, -1), y, R=R, S=R, stride=1, pad=pad)
torch.cuda.synchronize()
print("ok")
