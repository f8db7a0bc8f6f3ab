"""ZeRO-1 / ZeRO-2 sharded optimizer over flat fp32 buffers.

The reference ships DeepSpeed ZeRO configs (`/root/reference/02_deepspeed/deepspeed_config.py:53-105`:
stage 1 with ``overlap_comm``, ``contiguous_gradients``, ``reduce_scatter`` and 5e8 buckets; stage
2; stage 3; stage 3 + CPU offload) but never passes them to DeepSpeed. Here
they are real:

* **stage 1** — gradients all-reduced as in DDP (bucketed, overlapped), then each rank updates
  only ITS contiguous 1/world shard of the flat master with its shard of the optimizer state
  (momentum / Adam moments), then the shards are all-gathered back into the full master;
* **stage 2** — gradients are reduce-scattered instead (each rank only ever holds the summed
  gradient of its own shard), then the same shard update + all-gather.

Both are bit-compatible with plain data parallel + the same optimizer (tests/test_dist_cpu.py).
Stage 3 (parameter sharding) and CPU offload live in ``parallel/fsdp.py`` (the training engine
routes ``zero.stage=3`` / ``offload_*`` there). This flat-buffer optimizer serves the native ResNet
program, whose captured HIP graph needs resident full parameters: asked for stage 3 directly it
runs stage 2 with a warning (ResNet-50's 102 MB of fp32 params fit 288 GB of HBM ~2800 times).

The shard update runs the fused HIP optimizer kernels (ops.kernels.sgd_step / adam_step) on GPU
and their PyTorch references on CPU.
"""
from __future__ import annotations

import math
import warnings
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist

from ..ops import kernels as K
from .dist import host_sync_for_gloo


def shard_range(n: int, rank: int, world: int, align: int = 16) -> Tuple[int, int]:
    """Contiguous, 16-element aligned shard [lo, hi) of an n-element flat buffer."""
    per = (n + world - 1) // world
    per = (per + align - 1) // align * align
    lo = min(n, rank * per)
    return lo, min(n, lo + per)


class ZeroShardedOptimizer:
    """Optimizer step over a flat master buffer with sharded optimizer state.

    ``master`` / ``grad``: fp32 flat tensors (same length; the DDP/native trainers' buffers).
    ``optim``: object with fields name, lr, momentum, nesterov, weight_decay, betas, eps, grad_clip.
    ``grads_already_reduced``: stage 1 with grads all-reduced (summed) by the caller's buckets.
    """

    def __init__(self, master: torch.Tensor, grad: torch.Tensor, optim, stage: int = 1, process_group=None,
                 grad_scale: Optional[float] = None):
        if stage not in (1, 2, 3):
            raise ValueError("ZeRO stage must be 1, 2 or 3")
        if optim.name not in ("sgd", "adam", "adamw"):
            raise ValueError(f"sharded optimizer supports sgd / adam / adamw, not {optim.name!r}")
        if stage == 3:
            warnings.warn("flat-buffer ZeRO: stage 3 runs as stage 2 here; parameter sharding is parallel.fsdp.ShardedDataParallel")
            stage = 2
        self.stage = stage
        self.master, self.grad, self.o = master, grad, optim
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_available() and dist.is_initialized() else 1
        self.rank = dist.get_rank(process_group) if self.world > 1 else 0
        n = master.numel()
        # pad the flat length to world * shard so all-gather / reduce-scatter see equal shards
        per = shard_range(n, 0, self.world)[1]
        self.per = per
        self.padded = per * self.world
        self.lo, self.hi = self.rank * per, min(n, (self.rank + 1) * per)
        dev = master.device
        self.m = torch.zeros(per, device=dev)
        self.v = torch.zeros(per, device=dev) if optim.name in ("adam", "adamw") else None
        self.step_count = 0
        self.grad_scale = grad_scale if grad_scale is not None else 1.0 / self.world
        self._gshard = torch.zeros(per, device=dev)
        self._pshard = torch.zeros(per, device=dev)
        self._clip = torch.zeros(4, device=dev)

    def shard_of(self, t: torch.Tensor) -> torch.Tensor:
        return t[self.lo:self.hi]

    def _padded_view(self, t: torch.Tensor) -> torch.Tensor:
        if t.numel() == self.padded:
            return t
        out = torch.zeros(self.padded, device=t.device, dtype=t.dtype)
        out[:t.numel()].copy_(t)
        return out

    @torch.no_grad()
    def step(self, grads_already_reduced: bool = True, lr: Optional[float] = None,
             hyper: Optional[torch.Tensor] = None):
        """``hyper``: optional fp32 device tensor (lr, 1-b1^t, 1-b2^t) read by the kernels at run
        time. The native trainer passes its own so a graph-captured step follows LR schedules and
        Adam bias correction on every replay (host scalars would be frozen at capture)."""
        o = self.o
        self.step_count += 1
        n_own = self.hi - self.lo
        g = self._gshard
        g.zero_()
        if self.world > 1:
            host_sync_for_gloo(self.grad, self.pg)
        if self.world == 1:
            g[:n_own].copy_(self.grad[self.lo:self.hi])
        elif self.stage == 1 or grads_already_reduced:
            if not grads_already_reduced:
                dist.all_reduce(self.grad, group=self.pg)
            g[:n_own].copy_(self.grad[self.lo:self.hi])
        else:
            full = self._padded_view(self.grad)
            try:
                dist.reduce_scatter_tensor(g, full, group=self.pg)
            except (RuntimeError, NotImplementedError, AttributeError):
                dist.all_reduce(full, group=self.pg)
                g.copy_(full[self.rank * self.per:(self.rank + 1) * self.per])
        p = self._pshard
        p.zero_()
        p[:n_own].copy_(self.master[self.lo:self.hi])
        gsp = None
        if getattr(o, "grad_clip", 0.0):
            # global norm over all shards: local sum of squares, all-reduced
            local = (g[:n_own] * self.grad_scale).float().pow(2).sum()
            if self.world > 1:
                host_sync_for_gloo(local, self.pg)
                dist.all_reduce(local, group=self.pg)
            self._clip[2] = torch.clamp(o.grad_clip / (local.sqrt() + 1e-6), max=1.0)
            gsp = self._clip[2:3]
        lr = o.lr if lr is None else lr
        if o.name == "sgd":
            K.sgd_step(p, g, self.m, None, lr=lr, momentum=o.momentum, dampening=getattr(o, "dampening", 0.0),
                       weight_decay=o.weight_decay, nesterov=o.nesterov, first=False, grad_scale_ptr=gsp,
                       grad_scale=self.grad_scale, hyper=hyper)
        else:
            K.adam_step(p, g, self.m, self.v, None, lr=lr, beta1=o.betas[0], beta2=o.betas[1], eps=o.eps,
                        weight_decay=o.weight_decay, decoupled=(o.name == "adamw"), step=self.step_count,
                        grad_scale_ptr=gsp, grad_scale=self.grad_scale, hyper=hyper)
        if self.world == 1:
            self.master[self.lo:self.hi].copy_(p[:n_own])
            return
        full = torch.empty(self.padded, device=p.device, dtype=p.dtype)
        host_sync_for_gloo(p, self.pg)
        dist.all_gather_into_tensor(full, p, group=self.pg)
        self.master.copy_(full[:self.master.numel()])

    def state_dict(self):
        return {"stage": self.stage, "step": self.step_count, "rank": self.rank, "world": self.world,
                "m": self.m.cpu(), "v": None if self.v is None else self.v.cpu()}

    def load_state_dict(self, sd):
        if sd["world"] != self.world:
            raise ValueError("ZeRO optimizer state was saved with a different world size")
        self.step_count = sd["step"]
        self.m.copy_(sd["m"])
        if self.v is not None and sd["v"] is not None:
            self.v.copy_(sd["v"])
