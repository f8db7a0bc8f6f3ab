#!/usr/bin/env python3
"""Which parameters' gradients differ between fused / unfused split-K wgrad reduction, graph / eager."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dbx_distributed_pytorch_examples_amd.engine.native_trainer import NativeTrainer, OptimConfig  # noqa: E402
from dbx_distributed_pytorch_examples_amd.models import build_model  # noqa: E402

arch = sys.argv[1] if len(sys.argv) > 1 else "cifar_resnet18"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 64
torch.manual_seed(0)
m = build_model(arch, num_classes=10)
trs = {}
for name, fuse, graphs in (("fg", "1", True), ("ug", "0", True), ("fe", "1", False), ("ue", "0", False)):
    os.environ["DBX_FUSE_WGRAD_REDUCE"] = fuse
    trs[name] = NativeTrainer(copy.deepcopy(m), B, (32, 32), torch.device("cuda"), optim=OptimConfig(lr=0.05),
                              use_graphs=graphs)
ranges = trs["fg"].prog.param_ranges
g = torch.Generator().manual_seed(1)
for i in range(4):
    img = torch.randint(0, 256, (B, 32, 32, 3), dtype=torch.uint8, generator=g).cuda()
    lab = torch.randint(0, 10, (B,), generator=g).cuda()
    for t in trs.values():
        t.step(img, lab)
    torch.cuda.synchronize()
    ref = trs["ue"].prog.grad
    for name in ("fg", "ug", "fe"):
        gr = trs[name].prog.grad
        bad = []
        for pn, off, n in ranges:
            a, b = gr[off:off + n], ref[off:off + n]
            if not torch.equal(a, b):
                bad.append(f"{pn}:{((a - b).norm() / b.norm().clamp_min(1e-30)).item():.1e}")
        print(f"step {i} {name} vs ue: {len(bad)} differing tensors {bad[:8]}", flush=True)
    print(f"step {i} cnt sum fused: {int(trs['fg'].prog.wg_cnt.abs().sum())} {int(trs['fe'].prog.wg_cnt.abs().sum())}")
