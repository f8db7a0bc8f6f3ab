"""Tracing / profiling (SURVEY §5.1 MI355X plan).

The reference has no profiler at all: wall-clock ``Timer`` around ``distributor.run``
(`utils/hf_dataset_utilities.py:83-89`, use `01_torch_distributor/02_cifar…:333-357`), ``nvidia-smi``
cells, and an unused DeepSpeed ``wall_clock_breakdown`` flag (`02_deepspeed/deepspeed_config.py:42-48`).
This module provides the MI355X equivalents:

* ``range(name)``: roctx ranges (``libroctx64``) so phases show up in ``rocprofv3 --marker-trace``;
  a no-op when the library is missing (CPU containers).
* ``PhaseTimer``: hipEvent (``torch.cuda.Event``) timing of named step phases, aggregated to
  mean/min/max milliseconds; CPU fallback uses ``perf_counter``.
* ``rocprof_cmd()``: the rocprofv3 command line for a kernel-trace + stats run, or a PMC
  counter run (kept separate: counters are never combined with sys/runtime traces on this pool).
* ``summarize_kernel_stats()`` / CLI ``python -m dbx_distributed_pytorch_examples_amd.utils.profiling
  summarize <dir>``: top-N kernels per step from a ``*_kernel_stats.csv``; ``counters`` derives
  MFMA busy %, VALU/MFMA ratio and LDS bank-conflict cycles from a ``counter_collection.csv``.
"""
from __future__ import annotations

import argparse
import contextlib
import csv
import ctypes
import glob
import os
import sys
import time
from collections import defaultdict
from typing import Dict, List, Optional, Sequence

import torch

_ROCTX = None
_ROCTX_TRIED = False

# counter groups that fit one pass each (rocprofv3 --pmc); see tools/gpu/pmc_step.sh
PMC_GROUPS = {
    "mfma": ["SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_VALU", "SQ_INSTS_MFMA",
             "SQ_INSTS_LDS"],
    "stalls": ["SQ_LDS_BANK_CONFLICT", "SQ_WAIT_INST_LDS", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_INSTS_VMEM_RD",
               "TA_BUSY_avr"],
}


def _roctx():
    global _ROCTX, _ROCTX_TRIED
    if not _ROCTX_TRIED:
        _ROCTX_TRIED = True
        for name in ("libroctx64.so", "/opt/rocm/lib/libroctx64.so"):
            try:
                lib = ctypes.CDLL(name)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.restype = ctypes.c_int
                lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                _ROCTX = lib
                break
            except (OSError, AttributeError):
                continue
    return _ROCTX


def roctx_available() -> bool:
    return _roctx() is not None


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors nvtx.range / roctx range naming
    """roctx range around a code region (visible in rocprofv3 --marker-trace)."""
    lib = _roctx() if "noroctx" not in os.environ.get("DBX_PROFILE", "").split(",") else None
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib is not None:
            lib.roctxRangePop()


def mark(name: str) -> None:
    lib = _roctx()
    if lib is not None:
        lib.roctxMarkA(name.encode())


class PhaseTimer:
    """Per-phase device time of a training step (data / fwd / bwd / comm-wait / opt ...).

    ``with t.phase("fwd"): ...`` records a pair of events on the current stream; ``summary()``
    synchronizes once and returns {phase: {"mean_ms", "min_ms", "max_ms", "count"}}.
    """

    def __init__(self, enabled: bool = True, use_cuda: Optional[bool] = None):
        self.enabled = enabled
        self.use_cuda = torch.cuda.is_available() if use_cuda is None else use_cuda
        self._pending: List = []
        self._ms: Dict[str, List[float]] = defaultdict(list)

    @contextlib.contextmanager
    def phase(self, name: str):
        if not self.enabled:
            yield
            return
        with range(name):
            if self.use_cuda:
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                try:
                    yield
                finally:
                    e.record()
                    self._pending.append((name, s, e))
            else:
                t0 = time.perf_counter()
                try:
                    yield
                finally:
                    self._ms[name].append(1000.0 * (time.perf_counter() - t0))

    def _flush(self):
        if self._pending:
            torch.cuda.synchronize()
            for name, s, e in self._pending:
                self._ms[name].append(s.elapsed_time(e))
            self._pending = []

    def summary(self) -> Dict[str, Dict[str, float]]:
        self._flush()
        return {k: {"mean_ms": sum(v) / len(v), "min_ms": min(v), "max_ms": max(v), "count": len(v)}
                for k, v in self._ms.items() if v}

    def reset(self):
        self._pending, self._ms = [], defaultdict(list)


def rocprof_cmd(program: Sequence[str], out_dir: str, pmc: Optional[Sequence[str]] = None,
                output_name: str = "run") -> List[str]:
    """rocprofv3 command line. The program goes directly after ``--`` (no env/bash wrapper:
    the profiler's preload initialises the GPU, so an exec hop would be a forbidden exec).
    ``pmc``: counter names for a counter-only pass (kernel trace implied); else kernel trace + stats."""
    cmd = ["rocprofv3"]
    if pmc:
        cmd += ["--pmc", *pmc]
    else:
        cmd += ["--kernel-trace", "--stats"]
    cmd += ["-d", out_dir, "-o", output_name, "--output-format", "csv", "--", *program]
    return cmd


def summarize_kernel_stats(path: str, steps: int = 1, top: int = 25) -> List[Dict]:
    """Rows of a rocprofv3 ``*_kernel_stats.csv`` → [{name, calls, ms_per_step, pct}] sorted."""
    if os.path.isdir(path):
        found = glob.glob(os.path.join(path, "**", "*kernel_stats.csv"), recursive=True)
        if not found:
            raise FileNotFoundError(f"no *kernel_stats.csv under {path}")
        path = found[0]
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows) or 1.0
    out = [{"name": r["Name"], "calls": int(r["Calls"]) / steps,
            "ms_per_step": float(r["TotalDurationNs"]) / 1e6 / steps,
            "pct": 100.0 * float(r["TotalDurationNs"]) / tot} for r in rows]
    out.sort(key=lambda d: -d["ms_per_step"])
    return out[:top]


def summarize_counters(path: str, match: str = "") -> Dict[str, Dict[str, float]]:
    """Aggregate a ``*counter_collection.csv`` per kernel and derive utilisation ratios."""
    if os.path.isdir(path):
        path = glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True)[0]
    agg: Dict[str, Dict[str, float]] = defaultdict(lambda: defaultdict(float))
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if match and match not in k:
            continue
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    out = {}
    for k, d in agg.items():
        dd = dict(d)
        if d.get("SQ_BUSY_CYCLES") and "SQ_VALU_MFMA_BUSY_CYCLES" in d:
            dd["mfma_busy_per_busy"] = d["SQ_VALU_MFMA_BUSY_CYCLES"] / d["SQ_BUSY_CYCLES"]
        if d.get("SQ_INSTS_MFMA"):
            dd["valu_per_mfma"] = d.get("SQ_INSTS_VALU", 0.0) / d["SQ_INSTS_MFMA"]
        if d.get("SQ_INSTS_LDS") and "SQ_LDS_BANK_CONFLICT" in d:
            dd["lds_conflict_cycles_per_inst"] = d["SQ_LDS_BANK_CONFLICT"] / d["SQ_INSTS_LDS"]
        out[k] = dd
    return out


def _main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="dbx-profiling")
    sub = ap.add_subparsers(dest="cmd", required=True)
    s = sub.add_parser("summarize", help="top kernels from a rocprofv3 --stats output dir")
    s.add_argument("path")
    s.add_argument("--steps", type=int, default=1)
    s.add_argument("--top", type=int, default=25)
    c = sub.add_parser("counters", help="derived ratios from a rocprofv3 --pmc output dir")
    c.add_argument("path")
    c.add_argument("--match", default="")
    m = sub.add_parser("cmd", help="print the rocprofv3 command for a program")
    m.add_argument("--out", default="gpurun_out/prof")
    m.add_argument("--pmc", default="", help=f"counter group {sorted(PMC_GROUPS)} or comma list")
    m.add_argument("program", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    if a.cmd == "summarize":
        for r in summarize_kernel_stats(a.path, a.steps, a.top):
            print(f"{r['ms_per_step']:9.3f} ms {r['calls']:7.1f} calls {r['pct']:5.1f}%  {r['name'][:110]}")
    elif a.cmd == "counters":
        for k, d in summarize_counters(a.path, a.match).items():
            print(k[:100])
            print("   ", {n: (round(v, 4) if isinstance(v, float) else v) for n, v in d.items()})
    else:
        pmc = PMC_GROUPS.get(a.pmc, [x for x in a.pmc.split(",") if x])
        prog = a.program[1:] if a.program and a.program[0] == "--" else a.program
        print(" ".join(rocprof_cmd(prog, a.out, pmc or None)))
    return 0


if __name__ == "__main__":
    sys.exit(_main())
