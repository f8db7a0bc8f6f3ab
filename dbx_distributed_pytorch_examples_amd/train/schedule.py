"""Learning-rate schedules (host-side; the value is pushed to the device each step so captured
graphs follow it).

Covers the reference's schedules — Accelerate's ``CosineAnnealingLR(T_max=epochs)`` stepped per
epoch (`04_accelerate/01_cifar_accelerate.ipynb:482-487`, `:671`) and DeepSpeed's ``WarmupLR``
(`02_deepspeed/deepspeed_config.py:33-40`) — plus the large-batch recipe the north-star 8192-batch
config needs (linear scaling rule + warmup, then cosine/linear decay).
"""
from __future__ import annotations

import math


def linear_scaled_lr(base_lr: float, global_batch: int, reference_batch: int = 256) -> float:
    """Goyal et al. linear scaling: lr = base * global_batch / 256."""
    return base_lr * global_batch / reference_batch


class LRSchedule:
    def __init__(self, name: str, base_lr: float, total_steps: int = 0, warmup_steps: int = 0,
                 warmup_min_lr: float = 0.0, steps_per_epoch: int = 1, t_max_epochs: int = 0,
                 step_size: int = 30, gamma: float = 0.1, min_lr: float = 0.0, warmup_type: str = "log"):
        self.name = name
        self.base = base_lr
        self.total = max(1, total_steps)
        self.warm = warmup_steps
        self.wmin = warmup_min_lr
        self.spe = max(1, steps_per_epoch)
        self.tmax = t_max_epochs
        self.step_size, self.gamma, self.min_lr = step_size, gamma, min_lr
        self.warmup_type = warmup_type

    def __call__(self, step: int) -> float:
        """LR for optimizer step ``step`` (0-based)."""
        if self.warm and step < self.warm:
            if self.name == "warmup_lr":  # DeepSpeed WarmupLR: log (default) or linear warmup, then constant
                if self.warmup_type == "linear":
                    frac = step / self.warm
                else:
                    frac = math.log(step + 1) / math.log(self.warm) if self.warm > 1 else 1.0
                return self.wmin + (self.base - self.wmin) * frac
            return self.base * (step + 1) / self.warm
        n = self.name
        if n in ("none", "constant", "warmup_lr", ""):
            return self.base
        if n == "cosine":  # per-epoch CosineAnnealingLR(T_max)
            e = step // self.spe
            T = self.tmax or max(1, self.total // self.spe)
            return self.min_lr + (self.base - self.min_lr) * (1 + math.cos(math.pi * min(e, T) / T)) / 2
        if n == "warmup_cosine":
            p = min(1.0, (step - self.warm) / max(1, self.total - self.warm))
            return self.min_lr + (self.base - self.min_lr) * (1 + math.cos(math.pi * p)) / 2
        if n == "warmup_linear":
            p = min(1.0, (step - self.warm) / max(1, self.total - self.warm))
            return self.base * (1 - p) + self.min_lr * p
        if n == "step":
            return self.base * self.gamma ** ((step // self.spe) // self.step_size)
        raise ValueError(f"unknown schedule {n!r}")


def from_config(sched_cfg, base_lr: float, total_steps: int, steps_per_epoch: int) -> LRSchedule:
    return LRSchedule(sched_cfg.name, base_lr, total_steps=sched_cfg.total_steps or total_steps,
                      warmup_steps=sched_cfg.warmup_steps, warmup_min_lr=sched_cfg.warmup_min_lr,
                      steps_per_epoch=steps_per_epoch, t_max_epochs=sched_cfg.t_max_epochs,
                      step_size=sched_cfg.step_size, gamma=sched_cfg.gamma,
                      warmup_type=getattr(sched_cfg, "warmup_type", "log"))
