#!/usr/bin/env python3
"""Multi-rank native training on GPU. On a one-GPU box the ranks share cuda:0 and talk over gloo
(DBX_DIST_BACKEND=gloo); on a multi-GPU node the same script runs on RCCL, one GPU per rank.

Checks (all on the segmented-graph + comm-stream path that world > 1 takes):
  1. the data-parallel gradient equals the sum of every rank's single-process gradient of its own
     batch (computed by a world-1 trainer on a one-rank subgroup, gathered and summed in rank
     order): bit-equal at world 2 (a 2-term fp32 sum is order-free), <= 1e-6 relative above;
  2. replicas stay bit-identical across ranks; the per-segment graph-captured path matches the
     eager path bit for bit;
  3. ZeRO-1 (reduce-scatter + sharded update + bf16 all-gather) matches plain data parallel.
  python -m dbx_distributed_pytorch_examples_amd.launch --nproc-per-node 2 tools/dist_gpu_check.py

World 1 (the one-GPU RCCL rehearsal): ``DBX_FORCE_PG=1 DBX_ENGINE=segmented_graphs=1`` under the launcher
creates a one-rank RCCL group and forces the segmented multi-rank path, so every RCCL-only branch
(c10d reduce_scatter_tensor / all_gather_into_tensor in parallel/zero.py, the comm-stream bucket
all-reduces, with the engine's comm=native the framework communicator and the one-graph step) executes;
the checks hold bit-exactly (every collective is an identity).
"""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dbx_distributed_pytorch_examples_amd.engine.native_trainer import NativeTrainer, OptimConfig  # noqa: E402
from dbx_distributed_pytorch_examples_amd.models import build_model  # noqa: E402
from dbx_distributed_pytorch_examples_amd.parallel import dist as ddist  # noqa: E402
from dbx_distributed_pytorch_examples_amd.utils import debug  # noqa: E402

B = 16


def batches(steps):
    g = torch.Generator().manual_seed(100 + info.rank)
    out = []
    for _ in range(steps):
        img = torch.randint(0, 256, (B, 32, 32, 3), dtype=torch.uint8, generator=g)
        lab = torch.randint(0, 10, (B,), generator=g)
        out.append((img.to(info.device), lab.to(info.device)))
    return out


def run(use_graphs, zero=0, steps=4, bucket_mb=1.0, pg=None, optim="sgd"):
    torch.manual_seed(0)
    m = build_model("resnet18", num_classes=10)
    opt = OptimConfig(lr=0.05) if optim == "sgd" else OptimConfig(name="adamw", lr=1e-3, weight_decay=0.01)
    tr = NativeTrainer(m, B, (32, 32), info.device, optim=opt, use_graphs=use_graphs,
                       bucket_cap_mb=bucket_mb, zero_stage=zero, process_group=pg)
    if COMM == "native" and pg is None and info.device.type == "cuda" and info.backend == "nccl":
        assert tr.ncomm is not None, "comm=native did not create the framework communicator"
    if zero:
        assert tr.zero.coll, "ZeRO did not take the collective (reduce-scatter / all-gather) path"
    for img, lab in batches(steps):
        tr.step(img, lab)
    tr.sync_master()  # ZeRO: every rank updated only its shard of the fp32 master
    if info.device.type == "cuda":
        torch.cuda.synchronize()
    loss, _ = tr.read_metrics()
    return tr, loss


def params(tr):
    return torch.cat([p.detach().reshape(-1) for p in tr.prog.model.parameters()]).clone()


info = ddist.init_distributed()
W = info.world_size
from dbx_distributed_pytorch_examples_amd.engine_config import EngineConfig  # noqa: E402
assert W >= 2 or (dist.is_initialized() and EngineConfig.current().segmented_graphs), \
    f"{info}: world 1 needs DBX_FORCE_PG=1 DBX_ENGINE=segmented_graphs=1 (under the launcher)"
exact = W <= 2
COMM = EngineConfig.current().comm

# 1. DP gradient == sum of per-rank single-process gradients (one step, eager)
singles = [dist.new_group([r]) for r in range(W)]
tr_local, _ = run(False, steps=1, pg=singles[info.rank])
assert tr_local.world == 1
g_local = tr_local.prog.grad.detach().clone()
del tr_local
gathered = [torch.empty_like(g_local) for _ in range(W)]
dist.all_gather(gathered, g_local)
g_sum = gathered[0].clone()
for t in gathered[1:]:
    g_sum += t
tr_dp, _ = run(False, steps=1)
g_dp = tr_dp.prog.grad.detach().clone()
del tr_dp
relg = ((g_dp - g_sum).norm() / g_sum.norm()).item()
assert (relg == 0.0) if exact else (relg < 1e-6), f"DP gradient != sum of per-rank gradients: {relg}"

# 2. graphs vs eager, replicas in sync
tr_g, loss = run(True)
w_graph = tr_g.prog.master.detach().clone()
del tr_g
debug.assert_replicas_in_sync([w_graph], what="master weights (graphs)")
tr_e, _ = run(False)
w_eager = tr_e.prog.master.detach().clone()
del tr_e
debug.assert_replicas_in_sync([w_eager], what="master weights (eager)")
rel = ((w_graph - w_eager).norm() / w_eager.norm()).item()
assert rel == 0.0, f"graph vs eager mismatch {rel} (training is bit-reproducible: fp64 statistics atomics)"

# 3. ZeRO-1 == DP (SGD and AdamW)
relz = {}
for optim in ("sgd", "adamw"):
    tr_z, _ = run(True, zero=1, optim=optim)
    w_zero = params(tr_z)  # the ZeRO flat layout is padded differently: compare the module's tensors
    del tr_z
    debug.assert_replicas_in_sync([w_zero], what=f"master weights (ZeRO-1 {optim})")
    tr_d, _ = run(True, zero=0, optim=optim)
    w_dp = params(tr_d)
    del tr_d
    relz[optim] = ((w_zero - w_dp).norm() / w_dp.norm()).item()
    assert (relz[optim] == 0.0) if exact else (relz[optim] < 1e-6), f"ZeRO-1 vs DP mismatch ({optim}) {relz[optim]}"
if info.rank == 0:
    print(f"dist_gpu_check OK: world={W} backend={info.backend} comm={COMM} loss={loss:.3f} grad-vs-sum={relg:.2e} "
          f"graph-vs-eager={rel:.2e} zero1-vs-dp sgd={relz['sgd']:.2e} adamw={relz['adamw']:.2e}", flush=True)
ddist.destroy()
