"""Collective failure detection: a hung or failed peer ends the job so the launcher can restart it.

SURVEY.md §5.3: the reference relies on NCCL's own timeout (30 min) and Databricks' job retries;
a rank that is alive but stops issuing collectives (a stuck data loader, a deadlocked thread, a
GPU that wedged) leaves its peers blocked inside a collective with no progress signal the
launcher's heartbeat watchdog can see -- the blocked ranks are the ones that stop beating, but
only long after the fact, and their queued RCCL kernels keep the device busy.

:class:`CommWatchdog` bounds every training step instead. The training loop brackets each step
with :meth:`step_begin` / :meth:`step_end`; a daemon thread polls, every ``poll_s``:

* every registered framework communicator's asynchronous error state (``ncclCommGetAsyncError``
  through ``NativeComm.async_error``: a peer that died or a transport failure shows up there while
  the kernels are still queued);
* the age of the step in flight on the host (collectives that block the caller: gloo, c10d waits,
  the metric all-reduces) and of the last step's completion event on the device (stream-ordered RCCL
  collectives return at once and hang on the GPU instead).

On an error, or a step older than ``timeout_s``, it aborts every registered communicator
(``ncclCommAbort``: their queued kernels return, the streams drain), aborts the c10d process group
where torch supports it, prints the reason and ends the process with :data:`EXIT_COMM_FAILURE`. The
launcher (``launch.Launcher``) sees a rank exit non-zero, stops the other ranks and, with
``max_restarts``, starts a new attempt that resumes from the latest checkpoint
(``train(resume="latest")`` / ``DBX_RESTART_COUNT``). The c10d group itself is created with the same
timeout (``parallel.dist.init_distributed``), so a blocked gloo / RCCL call also raises on its own.

``DBX_COMM_TIMEOUT`` (seconds, default 1800 as c10d) sets the bound; ``utils.fault`` kind
``comm_hang`` injects the failure (a rank keeps beating but never issues another collective).
"""
from __future__ import annotations

import os
import sys
import threading
import time
from typing import List, Optional

import torch

EXIT_COMM_FAILURE = 75


def comm_timeout_s() -> float:
    return float(os.environ.get("DBX_COMM_TIMEOUT", "1800"))


class CommWatchdog:
    def __init__(self, timeout_s: Optional[float] = None, poll_s: float = 0.25, comms: Optional[List] = None,
                 device: Optional[torch.device] = None, exit_fn=None):
        self.timeout = comm_timeout_s() if timeout_s is None else float(timeout_s)
        self.poll = poll_s
        self.comms = list(comms or [])
        self.device = device
        self._exit = exit_fn or os._exit
        self._lock = threading.Lock()
        self._host_t0: Optional[float] = None  # step in flight on the host since
        self._step = -1
        self._ev = None                         # last step's completion event (device) ...
        self._ev_t0 = 0.0                       # ... recorded at
        self._stop = threading.Event()
        self.fired: Optional[str] = None
        self._th = threading.Thread(target=self._loop, name="dbx-comm-watchdog", daemon=True)
        self._th.start()

    def register(self, comm) -> None:
        if comm is not None:
            with self._lock:
                self.comms = self.comms + [comm]

    def unregister(self, comm) -> None:
        """Stop polling ``comm`` (before it is closed: bench.py's rebuild on the c10d path)."""
        with self._lock:
            self.comms = [c for c in self.comms if c is not comm]

    def step_begin(self, step) -> None:
        """``step``: a step number, or a phase label (bench.py brackets "setup" / "warmup" / "timed")."""
        with self._lock:
            self._host_t0 = time.monotonic()
            self._step = step

    def step_end(self) -> None:
        ev = None
        if self.device is not None and self.device.type == "cuda":
            ev = torch.cuda.Event()
            ev.record()
        with self._lock:
            self._host_t0 = None
            if ev is not None and (self._ev is None or self._ev.query()):
                # keep the OLDEST incomplete event: a device hang is measured from its first step
                self._ev, self._ev_t0 = ev, time.monotonic()

    def close(self) -> None:
        with self._lock:  # nothing in flight any more: a late poll must not fire
            self._host_t0, self._ev = None, None
        self._stop.set()
        self._th.join(timeout=2 * self.poll + 1)

    # ------------------------------------------------------------------------------------------
    def check(self) -> Optional[str]:
        """The failure to act on now, if any (also usable without the thread, e.g. in tests)."""
        with self._lock:
            comms = self.comms  # (replaced, never mutated in place: a snapshot)
        for c in comms:
            try:
                code, msg = c.async_error()
            except Exception as e:  # noqa: BLE001 - an unreachable communicator is a failure too
                return f"communicator error state unreadable: {e}"
            if code not in (0, 7):  # ncclSuccess, ncclInProgress
                return f"RCCL async error {code}: {msg}"
        now = time.monotonic()
        with self._lock:
            t0, step, ev, et0 = self._host_t0, self._step, self._ev, self._ev_t0
        what = f"step {step}" if isinstance(step, int) else f"phase {step!r}"
        if t0 is not None and now - t0 > self.timeout:
            return f"{what} has not completed its collectives within {self.timeout:.0f}s (host)"
        if ev is not None and now - et0 > self.timeout and not ev.query():
            return f"device work of {what} has not completed within {self.timeout:.0f}s"
        return None

    def _loop(self) -> None:
        while not self._stop.wait(self.poll):
            why = self.check()
            if why is not None:
                self.fire(why)
                return

    def fire(self, why: str) -> None:
        self.fired = why
        rank = os.environ.get("RANK", "0")
        print(f"[comm-watchdog] rank {rank}: {why}; aborting communicators and exiting "
              f"(code {EXIT_COMM_FAILURE}) for the launcher to restart", file=sys.stderr, flush=True)
        for c in self.comms:
            try:
                c.abort()
            except Exception:  # noqa: BLE001
                pass
        try:
            import torch.distributed as dist
            abort = getattr(dist.distributed_c10d, "_abort_process_group", None)
            if abort is not None and dist.is_initialized() and dist.get_backend() == "nccl":
                abort()
        except Exception:  # noqa: BLE001
            pass
        self._exit(EXIT_COMM_FAILURE)


def for_runner(runner, device: torch.device) -> Optional[CommWatchdog]:
    """A watchdog for a training run at world > 1 (None at world 1 unless DBX_COMM_TIMEOUT is set),
    with the runner's framework communicators registered."""
    from . import dist as ddist
    if ddist.get_world_size() == 1 and "DBX_COMM_TIMEOUT" not in os.environ:
        return None
    wd = CommWatchdog(device=device)
    tr = getattr(runner, "tr", None)
    wd.register(getattr(tr, "ncomm", None))
    return wd
