"""Process-group bootstrap and small collective helpers.

Replaces the reference's five launcher-specific bootstraps (`dist.init_process_group("nccl")`
at `/root/reference/01_torch_distributor/01_basic_torch_distributor.py:268-272`, Accelerate's
`accelerator.prepare`, Ray's `prepare_model`, …) with one env:// rendezvous: one process per
GPU, ``RANK/LOCAL_RANK/WORLD_SIZE/MASTER_ADDR/MASTER_PORT`` from the launcher (ours or
torchrun), backend ``"nccl"`` (= RCCL on ROCm, over xGMI) when a GPU is present, ``gloo``
otherwise. Unlike the reference's ResNet paths (`02_cifar…:191`, which never call
``set_device``) the device is always pinned to ``LOCAL_RANK``.

Metric reductions use ONE packed all-reduce per call (the reference issues 3+3 0-d
``accelerator.gather`` calls per epoch, `04_accelerate/01_cifar_accelerate.ipynb:638-664`).
String/object broadcast goes through the c10d store-backed object collectives, not a padded
int tensor (`01_cifar_accelerate.ipynb:764-778`).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Any, List, Optional, Sequence

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    local_rank: int = 0
    world_size: int = 1
    local_world_size: int = 1
    backend: str = "none"
    device: torch.device = torch.device("cpu")

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    @property
    def distributed(self) -> bool:
        return self.world_size > 1


_INFO: Optional[DistInfo] = None


def env_int(name: str, default: int) -> int:
    v = os.environ.get(name)
    return int(v) if v not in (None, "") else default


def init_distributed(backend: Optional[str] = None, device: Optional[str] = None,
                     timeout_s: Optional[float] = None) -> DistInfo:
    """Initialise (idempotently) the default process group from env:// variables.

    ``timeout_s``: the c10d collective timeout (default ``DBX_COMM_TIMEOUT``, else 1800 s) -- a
    blocked collective raises after it (see ``parallel.comm_guard``).

    ``device``: "cuda" / "cpu" / None (auto). With world_size 1 and no MASTER_ADDR the
    process group is skipped entirely (pure single-process mode).
    """
    global _INFO
    if _INFO is not None and (not _INFO.distributed or dist.is_initialized()):
        return _INFO
    if timeout_s is None:
        timeout_s = float(os.environ.get("DBX_COMM_TIMEOUT", "1800"))
    rank = env_int("RANK", 0)
    world = env_int("WORLD_SIZE", 1)
    local_rank = env_int("LOCAL_RANK", 0)
    local_world = env_int("LOCAL_WORLD_SIZE", world)
    use_cuda = (device == "cuda") or (device is None and torch.cuda.is_available())
    if use_cuda:
        torch.cuda.set_device(local_rank % max(1, torch.cuda.device_count()))
        dev = torch.device("cuda", torch.cuda.current_device())
    else:
        dev = torch.device("cpu")
    if backend is None:
        # DBX_DIST_BACKEND=gloo lets several ranks share one GPU (RCCL refuses duplicate devices),
        # which is how the multi-rank GPU path is exercised on a single-GPU box
        backend = os.environ.get("DBX_DIST_BACKEND") or ("nccl" if use_cuda else "gloo")
    # DBX_FORCE_PG=1 (under a launcher) creates the process group even at world 1: a one-GPU box
    # can then rehearse the RCCL code path (tools/dist_gpu_check.py at world 1, tests/test_multirank_gpu.py)
    force_pg = os.environ.get("DBX_FORCE_PG", "0") == "1" and "MASTER_PORT" in os.environ
    if world > 1 or force_pg:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        if not dist.is_initialized():
            kw: dict = dict(backend=backend, init_method="env://", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=timeout_s))
            if backend == "nccl":
                kw["device_id"] = dev
            dist.init_process_group(**kw)
    else:
        backend = "none"
    _INFO = DistInfo(rank, local_rank, world, local_world, backend, dev)
    return _INFO


def host_sync_for_gloo(t: torch.Tensor, group=None) -> None:
    """gloo reads CUDA tensors through its own copies, which are not ordered after kernels queued on
    the caller's stream: drain that stream first (gloo-on-GPU is the single-GPU multi-rank test
    configuration; RCCL collectives are stream-ordered and never take this path)."""
    if t.is_cuda and dist.is_initialized() and dist.get_backend(group) == "gloo":
        torch.cuda.current_stream(t.device).synchronize()


def info() -> DistInfo:
    return _INFO if _INFO is not None else init_distributed()


def destroy() -> None:
    global _INFO
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
    _INFO = None


def is_dist() -> bool:
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def get_rank() -> int:
    return dist.get_rank() if is_dist() else 0


def get_world_size() -> int:
    return dist.get_world_size() if is_dist() else 1


def barrier() -> None:
    if is_dist():
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def all_reduce_sum(values: Sequence[float], device: Optional[torch.device] = None) -> List[float]:
    """Sum a small vector of python floats over ranks with ONE collective."""
    if not is_dist():
        return [float(v) for v in values]
    dev = device or info().device
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=dev)
    dist.all_reduce(t)
    return t.tolist()


def all_reduce_tensor_(t: torch.Tensor, op: str = "sum") -> torch.Tensor:
    if is_dist():
        dist.all_reduce(t, op={"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX,
                               "min": dist.ReduceOp.MIN}[op])
    return t


def all_reduce_max(x: float) -> float:
    if not is_dist():
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=info().device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def broadcast_object(obj: Any, src: int = 0) -> Any:
    if not is_dist():
        return obj
    lst = [obj]
    dist.broadcast_object_list(lst, src=src)
    return lst[0]


def broadcast_tensor_(t: torch.Tensor, src: int = 0) -> torch.Tensor:
    if is_dist():
        dist.broadcast(t, src=src)
    return t
