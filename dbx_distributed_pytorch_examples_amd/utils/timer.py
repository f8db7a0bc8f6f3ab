"""Timers: the reference's wall-clock ``Timer`` (`utils/hf_dataset_utilities.py:83-89`) plus
GPU-event step timers that do not synchronise the host every step."""
from __future__ import annotations

import time
import timeit
from typing import List, Optional


class Timer:
    """``t = Timer(); ...; elapsed = t.stop()`` (reference API)."""

    def __init__(self):
        self.start = timeit.default_timer()
        self.end: Optional[float] = None

    def stop(self) -> float:
        self.end = timeit.default_timer()
        return self.end - self.start


class StepTimer:
    """Records a HIP event pair per step; ``summary()`` resolves them once (one sync)."""

    def __init__(self, enabled: bool = True):
        import torch
        self.enabled = enabled and torch.cuda.is_available()
        self._events: List = []
        self._wall: List[float] = []
        self._t = None

    def begin(self):
        import torch
        if self.enabled:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self._events.append([e, None])
        self._t = time.perf_counter()

    def end(self):
        import torch
        if self.enabled and self._events and self._events[-1][1] is None:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self._events[-1][1] = e
        if self._t is not None:
            self._wall.append(time.perf_counter() - self._t)

    def summary(self) -> dict:
        import torch
        gpu = []
        if self.enabled and self._events:
            torch.cuda.synchronize()
            gpu = [a.elapsed_time(b) for a, b in self._events if b is not None]
        out = {"steps": len(self._wall)}
        if gpu:
            s = sorted(gpu)
            out.update(gpu_ms_mean=sum(gpu) / len(gpu), gpu_ms_p50=s[len(s) // 2], gpu_ms_max=s[-1])
        if self._wall:
            out["host_ms_mean"] = 1000 * sum(self._wall) / len(self._wall)
        return out
