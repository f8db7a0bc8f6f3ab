"""Framework-owned RCCL communicator (SURVEY.md §5.8 "comm backend").

The reference only reaches NCCL through c10d (`dist.init_process_group("nccl")`,
`/root/reference/01_torch_distributor/01_basic_torch_distributor.py:269`) and DDP's reducer.
:class:`NativeComm` drives RCCL directly through ``csrc/runtime/comm.cpp``:

* one communicator per process group, bootstrapped with a unique id that rank 0 of the group
  creates and shares over the group's c10d store-backed object broadcast (gloo or RCCL groups);
* collectives are enqueued on the CALLER's current HIP stream (the trainer's comm stream) with no
  c10d work object and no watchdog thread, so they can be recorded into a HIP graph next to
  the backward kernels that produce the buckets;
* bucketed all-reduce / reduce-scatter / all-gather / broadcast on flat tensors, with the
  average folded into RCCL (``ncclAvg``) instead of a separate scale kernel.

The process's RCCL library is the one torch loaded (resolved with ``dlopen(RTLD_NOLOAD)``), so
both paths share one RCCL instance. On CPU-only builds or gloo groups, :func:`native_comm_available`
is False and callers keep using ``torch.distributed``.
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.distributed as dist

_DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2, torch.float64: 3, torch.int32: 4, torch.int64: 5,
       torch.uint8: 6}
_OP = {"sum": 0, "avg": 1, "max": 2, "min": 3, "prod": 4}


def _C():
    from ..ops._ext import C
    return C()


def native_comm_available() -> bool:
    """RCCL loadable and a GPU present (the communicator is device-bound)."""
    if not torch.cuda.is_available():
        return False
    try:
        return bool(_C().comm_available())
    except Exception:
        return False


def native_comm_requested() -> bool:
    """The engine's multi-rank gradient collectives go through :class:`NativeComm` (one-graph step)
    unless ``DBX_COMM=torch`` (c10d collectives between per-segment graphs). Default native: over a
    world-1 RCCL group on one MI355X the one-graph step runs at the single-graph rate (ResNet-18 CIFAR
    230.9k vs 231.9k img/s, TinyImageNet 96.7k vs 96.5k, headline 16.29k vs 16.36k) where the c10d
    path loses 21 % / 12 % / 1.4 % (profiles/r4_s3/)."""
    return os.environ.get("DBX_COMM", "native") == "native"


def open_verified_comm(process_group=None, device: Optional[torch.device] = None) -> "Optional[NativeComm]":
    """A :class:`NativeComm` over ``process_group`` that has passed a check all-reduce and all-gather
    on every rank -- or None on EVERY rank (the caller keeps the c10d collectives) when the
    communicator cannot be created or returns wrong sums anywhere. The decision is itself agreed over
    the c10d group, so no rank takes the framework path while another falls back."""
    import warnings
    ok, nc, err = native_comm_available(), None, "RCCL not loadable"
    if ok:
        try:
            nc = NativeComm(process_group, device)
            ok, err = nc.verify(), "check collectives returned wrong values"
        except Exception as e:  # noqa: BLE001 -- any failure means: stay on c10d
            ok, nc, err = False, None, f"{type(e).__name__}: {e}"
    dev = device or torch.device("cuda", torch.cuda.current_device())
    flag = torch.tensor([1 if ok else 0], dtype=torch.int32,
                        device=dev if dist.get_backend(process_group) == "nccl" else "cpu")
    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=process_group)
    if int(flag.item()) == 1:
        return nc
    if not ok:
        warnings.warn(f"framework RCCL communicator unavailable ({err}): using c10d collectives")
    return None


def _stream_ptr(stream: Optional[torch.cuda.Stream]) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


class NativeComm:
    """An RCCL communicator over the ranks of ``process_group`` (default: the world).

    Every rank of the group must construct it collectively (the unique id is broadcast from the
    group's first rank, then ``ncclCommInitRank`` rendezvouses over RCCL's own bootstrap)."""

    def __init__(self, process_group=None, device: Optional[torch.device] = None):
        if not dist.is_initialized():
            raise RuntimeError("NativeComm needs an initialised torch.distributed process group for its bootstrap")
        self.pg = process_group
        self.size = dist.get_world_size(process_group)
        self.rank = dist.get_rank(process_group)
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        c = _C()
        obj = [c.comm_unique_id() if self.rank == 0 else None]
        src = dist.get_global_rank(process_group, 0) if process_group is not None else 0
        dist.broadcast_object_list(obj, src=src, group=process_group)
        with torch.cuda.device(self.device):
            self._h = c.comm_init(obj[0], self.size, self.rank)
        self._c = c

    def verify(self) -> bool:
        """Check collectives on the current stream (synchronised): an all-reduce of rank + 1 and an
        all-gather of the ranks must give the exact expected values on this rank."""
        t = torch.full((64,), float(self.rank + 1), device=self.device)
        self.all_reduce(t)
        g = torch.empty(self.size * 8, dtype=torch.int32, device=self.device)
        self.all_gather(g, torch.full((8,), self.rank, dtype=torch.int32, device=self.device))
        torch.cuda.synchronize(self.device)
        want = torch.arange(self.size, dtype=torch.int32).repeat_interleave(8)
        return bool((t.cpu() == self.size * (self.size + 1) / 2).all()) and torch.equal(g.cpu(), want)

    # ---- collectives (in place where the RCCL API allows it) -----------------------------------
    def all_reduce(self, t: torch.Tensor, op: str = "sum", stream=None) -> torch.Tensor:
        self._chk(t)
        self._c.comm_all_reduce(self._h, t.data_ptr(), t.data_ptr(), t.numel(), _DT[t.dtype], _OP[op],
                                _stream_ptr(stream))
        return t

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, op: str = "sum", stream=None) -> torch.Tensor:
        """``out`` (n) = reduction over ranks of ``inp[rank*n:(rank+1)*n]`` (``inp`` holds size*n)."""
        self._chk(out)
        self._chk(inp)
        if inp.numel() != out.numel() * self.size or inp.dtype != out.dtype:
            raise ValueError("reduce_scatter: input must hold world_size x output elements of the same dtype")
        self._c.comm_reduce_scatter(self._h, inp.data_ptr(), out.data_ptr(), out.numel(), _DT[out.dtype], _OP[op],
                                    _stream_ptr(stream))
        return out

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor, stream=None) -> torch.Tensor:
        """``out`` (size*n) = concatenation over ranks of ``inp`` (n); ``inp`` may alias its slot of ``out``."""
        self._chk(out)
        self._chk(inp)
        if out.numel() != inp.numel() * self.size or inp.dtype != out.dtype:
            raise ValueError("all_gather: output must hold world_size x input elements of the same dtype")
        self._c.comm_all_gather(self._h, inp.data_ptr(), out.data_ptr(), inp.numel(), _DT[inp.dtype],
                                _stream_ptr(stream))
        return out

    def broadcast(self, t: torch.Tensor, root: int = 0, stream=None) -> torch.Tensor:
        self._chk(t)
        self._c.comm_broadcast(self._h, t.data_ptr(), t.data_ptr(), t.numel(), _DT[t.dtype], root,
                               _stream_ptr(stream))
        return t

    def fused_group(self):
        """Context manager fusing the collectives issued inside into one RCCL launch group."""
        comm = self

        class _G:
            def __enter__(self_):
                comm._c.comm_group_start()

            def __exit__(self_, *exc):
                comm._c.comm_group_end()
        return _G()

    def async_error(self):
        """(code, message) of the communicator's asynchronous error state (``ncclCommGetAsyncError``):
        code 0 = healthy, 7 (``ncclInProgress``) = still initialising, -1 = aborted, else a failure."""
        if not getattr(self, "_h", 0):
            return -1, "communicator closed"
        code, msg = self._c.comm_async_error(self._h)
        return int(code), str(msg)

    def abort(self) -> None:
        """``ncclCommAbort`` (safe from another thread while this one waits on the device): queued
        collectives of this communicator return, so the streams drain; the communicator is unusable after."""
        if getattr(self, "_h", 0):
            self._c.comm_abort(self._h)

    def close(self, abort: bool = False) -> None:
        if getattr(self, "_h", 0):
            self._c.comm_destroy(self._h, abort)
            self._h = 0

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, t: torch.Tensor) -> None:
        if not t.is_cuda or not t.is_contiguous():
            raise ValueError("NativeComm collectives take contiguous device tensors")
        if t.dtype not in _DT:
            raise ValueError(f"NativeComm: unsupported dtype {t.dtype}")


def bus_bandwidth(op: str, nbytes: int, seconds: float, world: int) -> float:
    """nccl-tests bus bandwidth (GB/s): the per-link rate a ring of ``world`` ranks sustains."""
    algbw = nbytes / seconds / 1e9
    f = {"all_reduce": 2.0 * (world - 1) / world, "reduce_scatter": (world - 1) / world,
         "all_gather": (world - 1) / world, "broadcast": 1.0}[op]
    return algbw * f
