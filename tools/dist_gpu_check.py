#!/usr/bin/env python3
"""Multi-rank native training on GPU (world 2). On a one-GPU box both ranks share cuda:0 and talk
over gloo (DBX_DIST_BACKEND=gloo); on a multi-GPU node the same script runs on RCCL. Checks:
replicas stay bit-identical across ranks, the per-segment graph-captured path matches the eager
path bit for bit, ZeRO-1 matches plain data parallel bit for bit (every reduction in the step is
order-independent: fp64 statistics atomics, fixed-order split-K and shard sums).
  python -m dbx_distributed_pytorch_examples_amd.launch --nproc-per-node 2 tools/dist_gpu_check.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dbx_distributed_pytorch_examples_amd.engine.native_trainer import NativeTrainer, OptimConfig  # noqa: E402
from dbx_distributed_pytorch_examples_amd.models import build_model  # noqa: E402
from dbx_distributed_pytorch_examples_amd.parallel import dist as ddist  # noqa: E402
from dbx_distributed_pytorch_examples_amd.utils import debug  # noqa: E402


def run(use_graphs, zero=0, steps=4, bucket_mb=1.0):
    torch.manual_seed(0)
    m = build_model("resnet18", num_classes=10)
    tr = NativeTrainer(m, 16, (32, 32), info.device, optim=OptimConfig(lr=0.05), use_graphs=use_graphs,
                       bucket_cap_mb=bucket_mb, zero_stage=zero)
    g = torch.Generator().manual_seed(100 + info.rank)
    for _ in range(steps):
        img = torch.randint(0, 256, (16, 32, 32, 3), dtype=torch.uint8, generator=g)
        lab = torch.randint(0, 10, (16,), generator=g)
        tr.step(img.to(info.device), lab.to(info.device))
    torch.cuda.synchronize()
    loss, corr = tr.read_metrics()
    return tr.prog.master.detach().clone(), loss


info = ddist.init_distributed()
assert info.world_size == 2 or os.environ.get("DBX_FORCE_PG") == "1", info
w_graph, loss = run(True)
debug.assert_replicas_in_sync([w_graph], what="master weights (graphs)")
w_eager, _ = run(False)
debug.assert_replicas_in_sync([w_eager], what="master weights (eager)")
rel = ((w_graph - w_eager).norm() / w_eager.norm()).item()
assert rel == 0.0, f"graph vs eager mismatch {rel} (training is bit-reproducible: fp64 statistics atomics)"
w_zero, _ = run(True, zero=1)
debug.assert_replicas_in_sync([w_zero], what="master weights (ZeRO-1)")
relz = ((w_zero - w_eager).norm() / w_eager.norm()).item()
assert relz == 0.0, f"ZeRO-1 vs DP mismatch {relz}"
if info.rank == 0:
    print(f"dist_gpu_check OK: backend={info.backend} loss={loss:.3f} graph-vs-eager={rel:.2e} zero1-vs-dp={relz:.2e}",
          flush=True)
ddist.destroy()
