"""Per-step optimizer hyper-parameters (lr, Adam bias corrections) handed to the captured step graph.

The graph reads a small device tensor; the host refreshes it before each replay. The refresh must stay
cheap next to a ~1 ms launch-bound step (ResNet-18 CIFAR): no pinned allocation per step (a fresh
``pin_memory()`` each step was enough host work to let the GPU catch up with the graph submission), no
copy at all when the values did not change (SGD at a constant lr), and a small pinned ring whose slot is
rewritten only after its previous copy completed (the host may run steps ahead of the GPU).
"""
from __future__ import annotations

from typing import List, Optional

import torch


class DeviceHyper:
    def __init__(self, dev_tensor: torch.Tensor, slots: int = 4):
        self.t = dev_tensor
        self.cuda = dev_tensor.is_cuda
        self.slots = slots
        self._ring = None
        self._i = 0
        self._last: Optional[List[float]] = None

    def set(self, vals: List[float]) -> None:
        vals = [float(v) for v in vals]
        if vals == self._last:
            return
        self._last = vals
        src = torch.tensor(vals, dtype=torch.float32)
        if not self.cuda:
            self.t.copy_(src)
            return
        if self._ring is None:
            self._ring = [(torch.zeros(len(vals), dtype=torch.float32).pin_memory(), torch.cuda.Event())
                          for _ in range(self.slots)]
        buf, ev = self._ring[self._i]
        self._i = (self._i + 1) % self.slots
        ev.synchronize()  # this slot's previous copy has completed (a no-op for a fresh event)
        buf.copy_(src)
        self.t.copy_(buf, non_blocking=True)
        ev.record()

    def invalidate(self) -> None:
        """Force the next set() to copy (the device tensor was written elsewhere)."""
        self._last = None
