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

import datetime
import itertools
import os
import time
from typing import Callable, Optional

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


def native_comm_requested(cfg=None) -> bool:
    """The engine's multi-rank gradient collectives go through :class:`NativeComm` (one-graph step)
    unless the engine config says ``comm=torch`` (c10d collectives between per-segment graphs). Default native: over a
    world-1 RCCL group on one MI355X the one-graph step runs at the single-graph rate (ResNet-18 CIFAR
    230.9k vs 231.9k img/s, TinyImageNet 96.7k vs 96.5k, headline 16.29k vs 16.36k) where the c10d
    path loses 21 % / 12 % / 1.4 % (profiles/r4_s3/)."""
    from ..engine_config import EngineConfig
    return (cfg or EngineConfig.current()).comm == "native"


def comm_init_timeout() -> float:
    """Seconds the communicator bootstrap / check may take before the rank gives up
    (``DBX_COMM_INIT_TIMEOUT``, default 300)."""
    return float(os.environ.get("DBX_COMM_INIT_TIMEOUT", "300"))


class CommAgreementTimeout(RuntimeError):
    """A peer never reached an agreement point (it hung or died): the job must end (the launcher
    restarts it), not fall back alone."""


class _Agreement:
    """All-ranks decisions for one communicator bootstrap, kept off the GPU: every rank writes its
    vote into the c10d store (the TCPStore of the rendezvous) and waits, with a deadline, for every
    vote. A rank that fails early also posts a ``fail`` key that peers still inside a non-blocking
    RCCL init poll for, so they abort that init instead of waiting for the rank forever."""

    _gen = itertools.count()

    def __init__(self, process_group=None):
        self.pg = process_group
        self.rank = dist.get_rank(process_group)
        self.size = dist.get_world_size(process_group)
        ranks = dist.get_process_group_ranks(process_group) if process_group is not None else range(self.size)
        self.prefix = f"dbx/comm_agree/{'-'.join(str(r) for r in ranks)}/{next(self._gen)}/"
        try:
            self.store = dist.distributed_c10d._get_default_store()
        except Exception:  # noqa: BLE001 -- no store (custom init): agree with a c10d collective
            self.store = None

    def post_failure(self, why: str) -> None:
        if self.store is not None:
            self.store.set(self.prefix + "fail", f"rank {self.rank}: {why}")

    def peer_failed(self) -> bool:
        return self.store is not None and self.store.check([self.prefix + "fail"])

    def all_true(self, ok: bool, tag: str, timeout_s: float, device=None) -> bool:
        if self.store is None:
            dev = device if (device is not None and dist.get_backend(self.pg) == "nccl") else "cpu"
            flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.pg)
            return int(flag.item()) == 1
        self.store.set(f"{self.prefix}{tag}/{self.rank}", "1" if ok else "0")
        keys = [f"{self.prefix}{tag}/{r}" for r in range(self.size)]
        try:
            self.store.wait(keys, datetime.timedelta(seconds=timeout_s))
        except Exception as e:  # noqa: BLE001 -- the store raises on its deadline
            raise CommAgreementTimeout(f"rank {self.rank}: no agreement on {tag!r} within {timeout_s:.0f}s "
                                       f"(a peer hung or died): {e}") from e
        return all(self.store.get(k) == b"1" for k in keys)


def open_verified_comm(process_group=None, device: Optional[torch.device] = None,
                       timeout_s: Optional[float] = None) -> "Optional[NativeComm]":
    """A :class:`NativeComm` over ``process_group`` that passed its checks on every rank -- or None on
    EVERY rank (the caller keeps the c10d collectives).

    1. Every rank votes on :func:`native_comm_available` BEFORE anything is constructed.
    2. The communicator is created NON-blocking; while its rendezvous is in flight the rank polls its
       state and the agreement's ``fail`` key, and aborts the init when a peer failed or the deadline
       passes (a rank that raised can no longer leave its peers inside ``ncclCommInitRank``).
    3. Checks: an eager all-reduce + all-gather, then the same all-reduce CAPTURED in a HIP graph on a
       side stream forked from the capturing stream and joined back (the one-graph step's shape),
       replayed twice, every wait bounded.
    4. Every rank votes on the result; any failure anywhere -> every rank aborts its communicator and
       returns None. A peer that never votes -> :class:`CommAgreementTimeout` (the job ends, non-zero)."""
    import warnings
    timeout = comm_init_timeout() if timeout_s is None else float(timeout_s)
    ag = _Agreement(process_group)
    avail = native_comm_available()
    if not ag.all_true(avail, "available", timeout, device):
        if not avail:
            warnings.warn("framework RCCL communicator unavailable (RCCL not loadable): using c10d collectives")
        return None
    nc, ok, err = None, False, ""
    try:
        nc = NativeComm(process_group, device, blocking=False, timeout_s=timeout, abort_if=ag.peer_failed)
        ok = nc.verify(timeout)
        err = "" if ok else "check collectives returned wrong values"
        if ok:
            ok = nc.verify_captured(timeout)
            err = "" if ok else "captured check collective returned wrong values or timed out"
    except Exception as e:  # noqa: BLE001 -- any failure means: stay on c10d, on every rank
        ok, err = False, f"{type(e).__name__}: {e}"
    if not ok:
        ag.post_failure(err)
    if ag.all_true(ok, "verified", timeout, device):
        return nc
    if nc is not None:
        nc.close(abort=True)
    warnings.warn(f"framework RCCL communicator not used ({err or 'a peer failed its checks'}): "
                  "using c10d collectives")
    return None


def _stream_ptr(stream: Optional[torch.cuda.Stream]) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


class NativeComm:
    """An RCCL communicator over the ranks of ``process_group`` (default: the world).

    Every rank of the group must construct it collectively (the unique id is broadcast from the
    group's first rank, then ``ncclCommInitRank`` rendezvouses over RCCL's own bootstrap)."""

    def __init__(self, process_group=None, device: Optional[torch.device] = None, blocking: bool = True,
                 timeout_s: Optional[float] = None, abort_if: Optional[Callable[[], bool]] = None):
        if not dist.is_initialized():
            raise RuntimeError("NativeComm needs an initialised torch.distributed process group for its bootstrap")
        from .collective_plan import rccl_channel_bounds
        self.pg = process_group
        self.size = dist.get_world_size(process_group)
        self.rank = dist.get_rank(process_group)
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.direct = None  # DirectAllReduce once a buffer is registered (enable_direct)
        self.loopback = 0   # world-1 test aid: a sum all-reduce scales by this (the engine's comm_loopback)
        c = _C()
        obj = [c.comm_unique_id() if self.rank == 0 else None]
        src = dist.get_global_rank(process_group, 0) if process_group is not None else 0
        dist.broadcast_object_list(obj, src=src, group=process_group)
        lo, hi = rccl_channel_bounds(self.size)
        nonblocking = (not blocking) and bool(c.comm_config_supported())
        with torch.cuda.device(self.device):
            self._h = c.comm_init(obj[0], self.size, self.rank, 0 if nonblocking else 1, lo, hi)
        self._c = c
        from .comm_guard import comm_timeout_s
        c.comm_set_timeout(self._h, comm_timeout_s())  # bounds the wait on a collective's ncclInProgress
        if nonblocking:
            self._settle_init(comm_init_timeout() if timeout_s is None else float(timeout_s), abort_if)

    def _settle_init(self, timeout_s: float, abort_if) -> None:
        """Poll a non-blocking init until it completes; abort it when a peer failed or time runs out."""
        t0 = time.monotonic()
        while True:
            code, msg = self.async_error()
            if code == 0:
                return
            if code != 7:  # not ncclInProgress: the init failed
                self.close(abort=True)
                raise RuntimeError(f"ncclCommInitRank failed: {code} {msg}")
            if abort_if is not None and abort_if():
                self.close(abort=True)
                raise RuntimeError("a peer failed before the RCCL rendezvous completed")
            if time.monotonic() - t0 > timeout_s:
                self.close(abort=True)
                raise TimeoutError(f"RCCL rendezvous did not complete within {timeout_s:.0f}s")
            time.sleep(0.005)

    def _wait_device(self, timeout_s: float, stream=None) -> bool:
        """Wait (bounded) for the work queued so far on ``stream``; on timeout abort the communicator so
        its queued kernels return, and report False."""
        ev = torch.cuda.Event()
        ev.record(stream if stream is not None else torch.cuda.current_stream(self.device))
        t0 = time.monotonic()
        while not ev.query():
            if time.monotonic() - t0 > timeout_s:
                self.abort()
                return False
            time.sleep(0.0005)
        return True

    def verify(self, timeout_s: Optional[float] = None) -> bool:
        """Eager check collectives on the current stream: an all-reduce of rank + 1 and an all-gather
        of the ranks must give the exact expected values on this rank (bounded wait)."""
        timeout_s = comm_init_timeout() if timeout_s is None else timeout_s
        t = torch.full((64,), float(self.rank + 1), device=self.device)
        self.all_reduce(t)
        g = torch.empty(self.size * 8, dtype=torch.int32, device=self.device)
        self.all_gather(g, torch.full((8,), self.rank, dtype=torch.int32, device=self.device))
        if not self._wait_device(timeout_s):
            return False
        want = torch.arange(self.size, dtype=torch.int32).repeat_interleave(8)
        return bool((t.cpu() == self.size * (self.size + 1) / 2).all()) and torch.equal(g.cpu(), want)

    def verify_captured(self, timeout_s: Optional[float] = None, replays: int = 2) -> bool:
        """The one-graph step's pattern, checked: an all-reduce recorded into a HIP graph on a side stream
        forked from the capturing stream, main-stream work beside it, joined back, then a consumer of the
        reduced values; replayed ``replays`` times with fresh inputs, every wait bounded."""
        timeout_s = comm_init_timeout() if timeout_s is None else timeout_s
        dev = self.device
        want = float(self.size * (self.size + 1) // 2)
        x = torch.zeros(4096, device=dev)
        y = torch.zeros(4096, device=dev)
        side = torch.cuda.Stream(device=dev)
        cap = torch.cuda.Stream(device=dev)
        cap.wait_stream(torch.cuda.current_stream(dev))
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(cap):
            with torch.cuda.graph(g, stream=cap, capture_error_mode="thread_local"):
                cur = torch.cuda.current_stream(dev)
                side.wait_stream(cur)
                with torch.cuda.stream(side):
                    self.all_reduce(x, stream=side)
                y.add_(1.0)            # main-branch work next to the collective
                cur.wait_stream(side)  # join
                y.add_(x)              # consumer of the reduced values
        torch.cuda.current_stream(dev).wait_stream(cap)
        ok = True
        for it in range(replays):
            x.fill_(float(self.rank + 1))
            y.fill_(float(it))
            g.replay()
            if not self._wait_device(timeout_s):
                return False
            ok = ok and bool((x == want).all().item()) and bool((y == it + 1.0 + want).all().item())
        del g
        return ok

    # ---- collectives (in place where the RCCL API allows it) -----------------------------------
    def all_reduce(self, t: torch.Tensor, op: str = "sum", stream=None) -> torch.Tensor:
        self._chk(t)
        if self.loopback and self.size == 1 and op == "sum":
            with torch.cuda.stream(stream if stream is not None else torch.cuda.current_stream(self.device)):
                t.mul_(float(self.loopback))
            return t
        if op == "sum" and self.direct is not None and self.direct.takes(t):
            self.direct.all_reduce(t, stream)  # the plan chose the direct xGMI path for this range
            return t
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
                comm._c.comm_group_end(comm._h)
        return _G()

    def enable_direct(self, buf: torch.Tensor, grid: int = 64, timeout_s: Optional[float] = None) -> bool:
        """Register ``buf`` (the flat fp32 gradient buffer, same layout on every rank) for the direct
        two-shot all-reduce (``csrc/direct_ar.hip``); collective. Ranges of ``buf`` that the plan
        (``collective_plan.plan_allreduce``) sends down the direct path then take it in
        :meth:`all_reduce`. Every rank agrees, or none uses it."""
        import warnings
        timeout = comm_init_timeout() if timeout_s is None else float(timeout_s)
        ag = _Agreement(self.pg)
        d, err = None, ""
        try:
            # barrier deadlines well inside the verify wait: a missing peer ends the kernel (error bit,
            # poisoned range) before verify gives up, and the RCCL communicator is never aborted here
            d = DirectAllReduce(self, buf, grid=grid, barrier_timeout_s=max(0.05, timeout / 4), setup_timeout_s=timeout)
            ok = d.verify(timeout)
            err = "" if ok else "check all-reduce returned wrong values"
        except Exception as e:  # noqa: BLE001
            ok, err = False, f"{type(e).__name__}: {e}"
        if ag.all_true(ok, "direct", timeout, self.device):
            self.direct = d
            return True
        if d is not None:
            d.close()
        warnings.warn(f"direct xGMI all-reduce not used ({err or 'a peer failed its check'}): RCCL for every bucket")
        return False

    def async_error(self):
        """(code, message) of the communicator's asynchronous error state (``ncclCommGetAsyncError``):
        code 0 = healthy, 7 (``ncclInProgress``) = still initialising, -1 = aborted, else a failure."""
        if not getattr(self, "_h", 0):
            return -1, "communicator closed"
        d = getattr(self, "direct", None)
        if d is not None and d.pending_error():
            return -2, "direct xGMI all-reduce: a flag barrier timed out (a peer is missing); the range is NaN"
        code, msg = self._c.comm_async_error(self._h)
        return int(code), str(msg)

    def abort(self) -> None:
        """``ncclCommAbort`` (safe from another thread while this one waits on the device): queued
        collectives of this communicator return, so the streams drain; the communicator is unusable after."""
        if getattr(self, "_h", 0):
            self._c.comm_abort(self._h)

    def close(self, abort: bool = False) -> None:
        if getattr(self, "direct", None) is not None:
            self.direct.close()
            self.direct = None
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


class DirectAllReduce:
    """Direct two-shot all-reduce over peer-mapped (hipIPC) buffers, ``csrc/direct_ar.hip``.

    Construction is collective over ``comm``'s group: every rank exports the allocation holding
    ``buf`` and its flag array, receives every peer's handles (c10d object all-gather) and maps them.
    :meth:`takes` answers whether a tensor is an fp32 range of ``buf`` (the same offsets on every
    rank) that the plan sends down this path; :meth:`all_reduce` launches the kernel on the stream
    (capturable: the kernel's barrier generations live in device memory)."""

    def __init__(self, comm: "NativeComm", buf: torch.Tensor, grid: int = 64, barrier_timeout_s: float = 120.0,
                 setup_timeout_s: Optional[float] = None):
        from .collective_plan import DAR_MAX_RANKS
        if buf.dtype != torch.float32 or not buf.is_cuda or not buf.is_contiguous():
            raise ValueError("DirectAllReduce: a contiguous fp32 device buffer")
        if comm.size > DAR_MAX_RANKS:
            raise ValueError(f"DirectAllReduce: at most {DAR_MAX_RANKS} ranks (one xGMI mesh)")
        c = _C()
        self._c, self.comm, self.grid = c, comm, int(grid)
        self.buf, self.timeout = buf, float(barrier_timeout_s)
        self.rank, self.size = comm.rank, comm.size
        self._flags = self._gen = self._err = self._err_host = self._err_host_dev = 0
        self._opened = []
        # local setup (allocation, handle export) is voted on BEFORE the collective handle exchange, so
        # a rank that fails here cannot leave its peers blocked in all_gather_object
        mine, err = None, ""
        try:
            self._flags, self._gen, self._err, self._err_host, self._err_host_dev = c.dar_alloc(self.grid)
            h, off = c.ipc_handle(buf.data_ptr())
            fh, foff = c.ipc_handle(self._flags)
            mine = (h, off, fh, foff, buf.numel(), self.grid)
        except Exception as e:  # noqa: BLE001
            err = f"{type(e).__name__}: {e}"
        setup_timeout = comm_init_timeout() if setup_timeout_s is None else float(setup_timeout_s)
        if not _Agreement(comm.pg).all_true(mine is not None, "direct_setup", setup_timeout, comm.device):
            self.close()
            raise RuntimeError(f"DirectAllReduce: local setup failed on a rank ({err or 'a peer'})")
        allinfo = [None] * self.size
        dist.all_gather_object(allinfo, mine, group=comm.pg)
        self.peer_buf, self.peer_flags = [], []
        for r, (hr, offr, fhr, foffr, nr, gr) in enumerate(allinfo):
            if nr != buf.numel() or gr != self.grid:
                raise ValueError("DirectAllReduce: buffer size / grid differ between ranks")
            if r == self.rank:
                self.peer_buf.append(buf.data_ptr())
                self.peer_flags.append(self._flags)
                continue
            pb = c.ipc_open(hr)
            self._opened.append(pb)
            pf = c.ipc_open(fhr)
            self._opened.append(pf)
            self.peer_buf.append(pb + offr)
            self.peer_flags.append(pf + foffr)

    def in_buffer(self, t: torch.Tensor) -> bool:
        """An fp32 range of the registered buffer starting on a 16-byte boundary (the kernel's vectors)."""
        b0, p = self.buf.data_ptr(), t.data_ptr()
        return (t.dtype == torch.float32 and t.is_contiguous() and b0 <= p
                and p + 4 * t.numel() <= b0 + 4 * self.buf.numel() and (p - b0) % 16 == 0)

    def takes(self, t: torch.Tensor) -> bool:
        from .collective_plan import plan_allreduce
        return self.in_buffer(t) and plan_allreduce(t.numel(), 4, self.size, t.numel(),
                                                    allow_direct=True).path == "direct"

    def all_reduce(self, t: torch.Tensor, stream=None) -> None:
        off = t.data_ptr() - self.buf.data_ptr()
        self._c.dar_launch([b + off for b in self.peer_buf], list(self.peer_flags), self._gen, self._err,
                           t.numel(), self.rank, self.size, self.grid, self.timeout, _stream_ptr(stream),
                           self._err_host_dev)

    def errors(self) -> int:
        """The error word (bit 0: a flag barrier timed out); reading it synchronises the device."""
        torch.cuda.synchronize(self.comm.device)
        return int(self._c.dar_read_err(self._err, False))

    def pending_error(self) -> int:
        """The kernel's pinned host mirror of the error word, read WITHOUT a device sync (the comm
        watchdog's poll, through :meth:`NativeComm.async_error`): non-zero once any launch timed out."""
        return int(self._c.dar_host_err(self._err_host)) if self._err_host else 0

    def verify(self, timeout_s: float) -> bool:
        """A direct all-reduce of a buffer range holding rank + 1 must give the exact sum. The wait is on
        an event of this launch only: the kernel's own barrier deadlines (3 x ``self.timeout``, set
        below ``timeout_s`` by :meth:`NativeComm.enable_direct`) end it, so nothing is aborted here --
        in particular not the shared RCCL communicator the buckets fall back to."""
        n = min(self.buf.numel(), 1 << 16)
        saved = self.buf[:n].clone()
        self.buf[:n].fill_(float(self.rank + 1))
        self.all_reduce(self.buf[:n])
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.comm.device))
        t0 = time.monotonic()
        while not ev.query():
            if time.monotonic() - t0 > timeout_s:
                return False
            time.sleep(0.0005)
        ok = bool((self.buf[:n] == float(self.size * (self.size + 1) // 2)).all().item()) and self.errors() == 0
        self.buf[:n].copy_(saved)
        return ok

    def close(self) -> None:
        for p in self._opened:
            try:
                self._c.ipc_close(p)
            except Exception:  # noqa: BLE001
                pass
        self._opened = []
        if getattr(self, "_flags", 0):
            self._c.dar_free(self._flags, self._gen, self._err, self._err_host)
            self._flags = self._gen = self._err = self._err_host = self._err_host_dev = 0


def bus_bandwidth(op: str, nbytes: int, seconds: float, world: int) -> float:
    """nccl-tests bus bandwidth (GB/s): the per-link rate a ring of ``world`` ranks sustains."""
    algbw = nbytes / seconds / 1e9
    f = {"all_reduce": 2.0 * (world - 1) / world, "reduce_scatter": (world - 1) / world,
         "all_gather": (world - 1) / world, "broadcast": 1.0}[op]
    return algbw * f
