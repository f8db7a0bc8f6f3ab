"""Failure detection hooks used by the training loops (SURVEY.md §5.3 plan).

* :func:`heartbeat` — progress beacon: touches ``$DBX_HEARTBEAT_DIR/rank<r>`` (set by
  ``launch.Launcher``); the launcher's watchdog kills the job when a rank stops advancing.
* :func:`maybe_inject` — deterministic fault injection for tests: ``DBX_FAULT="rank:step:kind"``
  with kind ``exit`` (os._exit(3)), ``raise`` (RuntimeError), ``hang`` (sleep forever),
  ``nan`` (returns True so the caller poisons its loss), ``comm_hang`` (keeps beating but never
  issues another collective: the peers' ``parallel.comm_guard`` watchdog must end the job), ``diverge``
  (consumed by ``bench.py``: the rank perturbs its parameters after warm-up, and the replica check
  must refuse to report). Only fires on the attempt given as an optional fourth field
  (``"rank:step:kind:attempt"``, default 0) so a restarted job can run clean.
* :func:`check_finite` — cross-rank divergence / NaN guard (one all-reduce of a flag).
"""
from __future__ import annotations

import os
import time
from typing import Optional


def _rank() -> int:
    return int(os.environ.get("RANK", "0"))


def heartbeat(step: Optional[int] = None) -> None:
    d = os.environ.get("DBX_HEARTBEAT_DIR")
    if not d:
        return
    path = os.path.join(d, f"rank{_rank()}")
    try:
        with open(path, "w") as f:
            f.write(str(step if step is not None else time.time()))
    except OSError:
        pass


def parse_fault(spec: Optional[str] = None):
    spec = spec if spec is not None else os.environ.get("DBX_FAULT", "")
    if not spec:
        return None
    parts = spec.split(":")
    return int(parts[0]), int(parts[1]), parts[2]


def fault_attempt(spec: Optional[str] = None) -> int:
    spec = spec if spec is not None else os.environ.get("DBX_FAULT", "")
    parts = spec.split(":")
    return int(parts[3]) if len(parts) > 3 else 0


def maybe_inject(step: int) -> bool:
    f = parse_fault()
    if f is None:
        return False
    r, s, kind = f
    if int(os.environ.get("DBX_RESTART_COUNT", "0")) != fault_attempt():
        return False
    if r != _rank() or s != step:
        return False
    if kind == "exit":
        os._exit(3)
    if kind == "raise":
        raise RuntimeError(f"injected fault at rank {r} step {s}")
    if kind == "hang":
        while True:
            time.sleep(60)
    if kind == "comm_hang":
        while True:  # alive to the heartbeat watchdog, silent to the collectives
            heartbeat(step)
            time.sleep(0.5)
    if kind in ("nan", "diverge"):
        return kind == "nan"
    raise ValueError(f"unknown fault kind {kind!r}")


def check_finite(value: float) -> bool:
    """True iff ``value`` is finite on every rank (one tiny all-reduce when distributed)."""
    import math

    from ..parallel import dist as ddist
    bad = 0.0 if math.isfinite(value) else 1.0
    return ddist.all_reduce_sum([bad])[0] == 0.0
