"""Debug aids / race and divergence detection (SURVEY §5.2 MI355X plan).

The reference's only debug aids are env flags set unconditionally (`setup/00_setup.py:66-67`:
``CUDA_LAUNCH_BLOCKING=1``, ``TORCH_DISTRIBUTED_DEBUG=DETAIL``) plus NCCL debug exports in a
``%sh`` cell that never reach Python (`00_setup.py:117-123`). Here everything is opt-in:

* ``debug_env(level)``: the env for a debug launch (``AMD_SERIALIZE_KERNEL=3``,
  ``HIP_LAUNCH_BLOCKING=1``, ``NCCL_DEBUG=INFO`` — RCCL honours it — and
  ``TORCH_DISTRIBUTED_DEBUG=DETAIL``); never applied by default (launch blocking is a perf bug).
* ``DBX_DEBUG=1``: ``ops.kernels`` then synchronizes after every native kernel and raises with the
  op name on a HIP error or on non-finite outputs (``checked_op``); bounds are already validated
  on the host before every launch (``kernels._chk``).
* ``replica_checksum`` / ``assert_replicas_in_sync``: cross-rank parameter checksum assertion
  (detects DDP divergence, e.g. a rank that skipped an all-reduce).
* ``check_bucket_order``: DDP bucket ready-order checker — every rank must launch its gradient
  bucket all-reduces in the same order, or RCCL pairs mismatched buffers.
"""
from __future__ import annotations

import functools
import os
from typing import Dict, List, Optional, Sequence

import torch
import torch.distributed as dist


def enabled() -> bool:
    return os.environ.get("DBX_DEBUG", "0") not in ("", "0", "false", "False")


def debug_env(level: int = 1) -> Dict[str, str]:
    env = {"NCCL_DEBUG": "INFO", "TORCH_DISTRIBUTED_DEBUG": "DETAIL", "DBX_DEBUG": "1"}
    if level >= 2:
        env.update({"AMD_SERIALIZE_KERNEL": "3", "HIP_LAUNCH_BLOCKING": "1", "NCCL_DEBUG_SUBSYS": "INIT,COLL",
                    "TORCH_SHOW_CPP_STACKTRACES": "1"})
    return env


class KernelCheckError(RuntimeError):
    pass


def _outputs(res, args, kw) -> List[torch.Tensor]:
    if isinstance(res, torch.Tensor):
        return [res]
    if isinstance(res, (tuple, list)):
        return [r for r in res if isinstance(r, torch.Tensor)]
    return []


def checked_op(fn):
    """Wrap a native op: in debug mode, synchronize after it and validate outputs."""
    @functools.wraps(fn)
    def wrapper(*args, **kw):
        res = fn(*args, **kw)
        if enabled():
            dev_tensors = [a for a in list(args) + list(kw.values()) if isinstance(a, torch.Tensor) and a.is_cuda]
            if dev_tensors:
                try:
                    torch.cuda.synchronize()
                except RuntimeError as e:  # a kernel fault surfaces here, attributed to this op
                    raise KernelCheckError(f"{fn.__name__}: device error after launch: {e}") from e
                for t in _outputs(res, args, kw):
                    if t.is_floating_point() and not torch.isfinite(t.float()).all():
                        raise KernelCheckError(f"{fn.__name__}: non-finite values in output {tuple(t.shape)}")
        return res
    return wrapper


def replica_checksum(tensors: Sequence[torch.Tensor]) -> torch.Tensor:
    """Order-sensitive fp64 checksum (sum and weighted sum) of a list of tensors."""
    acc = torch.zeros(2, dtype=torch.float64, device=tensors[0].device if tensors else "cpu")
    for i, t in enumerate(tensors):
        v = t.detach().double().reshape(-1)
        w = 1.0 + (torch.arange(v.numel(), device=v.device, dtype=torch.float64) % 13) / 13.0 + (i % 7)
        acc[0] += v.sum()
        acc[1] += (v * w).sum()
    return acc


def assert_replicas_in_sync(tensors: Sequence[torch.Tensor], group=None, rtol: float = 1e-6,
                            what: str = "parameters") -> None:
    """All ranks must hold identical replicas (after an optimizer step in DP)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return
    c = replica_checksum(tensors)
    if dist.get_backend(group) == "nccl" and not c.is_cuda:
        c = c.cuda()
    allc = [torch.zeros_like(c) for _ in range(dist.get_world_size(group))]
    dist.all_gather(allc, c, group=group)
    ref = allc[0]
    for r, x in enumerate(allc):
        if not torch.allclose(x, ref, rtol=rtol, atol=0.0):
            raise AssertionError(f"{what} diverged: rank {r} checksum {x.tolist()} != rank 0 {ref.tolist()}")


def check_bucket_order(order: Sequence[int], group=None) -> None:
    """Every rank must have launched its DDP bucket all-reduces in the same order."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return
    gathered: List[Optional[List[int]]] = [None] * dist.get_world_size(group)
    dist.all_gather_object(gathered, list(order), group=group)
    for r, o in enumerate(gathered):
        if o != gathered[0]:
            raise AssertionError(f"DDP bucket order differs: rank {r} {o} vs rank 0 {gathered[0]}")
