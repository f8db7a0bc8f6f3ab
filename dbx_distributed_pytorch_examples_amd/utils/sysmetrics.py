"""GPU system metrics (the reference relies on MLflow system metrics + the Databricks cluster UI,
`02_cifar_torch_distributor_resnet.py:186`, `assets/gpu_utilization.png`). Samples
``rocm-smi --json`` (utilisation %, VRAM used) in a daemon thread and forwards them to a
logger as ``system/gpu_<i>_utilization_percentage`` / ``system/gpu_<i>_memory_usage_megabytes``
(MLflow's own system-metric names)."""
from __future__ import annotations

import json
import shutil
import subprocess
import threading
import time
from typing import Callable, Dict, Optional


def sample_gpus() -> Dict[str, float]:
    exe = shutil.which("rocm-smi") or "/opt/rocm/bin/rocm-smi"
    try:
        out = subprocess.run([exe, "--showuse", "--showmemuse", "--showmeminfo", "vram", "--json"],
                             capture_output=True, text=True, timeout=10).stdout
        data = json.loads(out[out.index("{"):]) if "{" in out else {}
    except Exception:
        return {}
    res = {}
    for card, vals in data.items():
        if not card.startswith("card"):
            continue
        i = card[4:]
        for k, v in vals.items():
            try:
                fv = float(str(v).strip("%"))
            except ValueError:
                continue
            kl = k.lower()
            if "gpu use" in kl:
                res[f"system/gpu_{i}_utilization_percentage"] = fv
            elif "vram total used memory" in kl:
                res[f"system/gpu_{i}_memory_usage_megabytes"] = fv / 2 ** 20
            elif "memory allocated" in kl or "vram%" in kl:
                res[f"system/gpu_{i}_memory_usage_percentage"] = fv
    return res


class SystemMetricsLogger:
    def __init__(self, interval_s: float = 10.0, log_fn: Optional[Callable] = None):
        self.interval = interval_s
        self.log_fn = log_fn
        self._stop = threading.Event()
        self._t: Optional[threading.Thread] = None
        self.step = 0
        self.history = []

    def _loop(self):
        while not self._stop.is_set():
            m = sample_gpus()
            self.history.append((time.time(), m))
            if self.log_fn:
                for k, v in m.items():
                    try:
                        self.log_fn(k, v, self.step)
                    except Exception:
                        pass
            self.step += 1
            self._stop.wait(self.interval)

    def start(self):
        self._t = threading.Thread(target=self._loop, daemon=True)
        self._t.start()
        return self

    def stop(self):
        self._stop.set()
        if self._t:
            self._t.join(timeout=self.interval + 1)
