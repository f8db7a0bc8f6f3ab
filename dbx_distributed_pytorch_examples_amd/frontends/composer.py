"""Composer-style ``Trainer`` (`03_composer/01_cifar_composer_resnet.ipynb:406-436`).

``Trainer(model, optimizers, train_dataloader, eval_dataloader, max_duration="2ep",
algorithms=[LabelSmoothing(0.1), CutMix(1.0), ChannelsLast()], loggers=[MLFlowLogger(...)]).fit()``.
Algorithms map onto the engine: label smoothing -> the CE target, CutMix -> the batch-mixing step
(soft-label CE), ChannelsLast -> a no-op marker (every GPU path here is NHWC end to end, K19).
The model follows Composer's ``forward(batch)`` / ``loss(outputs, batch)`` convention
(``models.ComposerResNet50``); plain modules work too.

On GPUs a ``ComposerResNet50`` trains on the native HIP program at any world size: its inner ResNet
is wrapped by ``engine.native_module`` for the train loader's batch size and image size (CutMix's
soft targets and label smoothing stay torch ops on the logits; other batch sizes run the torch
module on the same parameters); at world > 1 the wrapped program averages its own gradients per
backward segment (overlapped with the backward), so the trainer's DDP only passes them through. The engine field ``native_frontends=0`` keeps the stock module (2.5x slower at the notebook's
b128 CIFAR shape, ``profiles/r2s5_native_module/``).
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Sequence

import torch
import torch.nn as nn

from ..config import parse_duration
from ..parallel import dist as ddist
from ..utils import mlflow_compat as mlflow
from ..engine_config import EngineConfig


class Algorithm:
    pass


class LabelSmoothing(Algorithm):
    def __init__(self, smoothing: float = 0.1):
        self.smoothing = smoothing


class CutMix(Algorithm):
    def __init__(self, alpha: float = 1.0, num_classes: Optional[int] = None):
        self.alpha, self.num_classes = alpha, num_classes


class ChannelsLast(Algorithm):
    """NHWC memory format — the framework's native layout; kept for API parity."""


class ComposerModel(nn.Module):
    """Base class with Composer's hooks."""

    def forward(self, batch):  # pragma: no cover - abstract
        raise NotImplementedError

    def loss(self, outputs, batch):  # pragma: no cover - abstract
        raise NotImplementedError


class MLFlowLogger:
    def __init__(self, experiment_name: str = "composer", tracking_uri: Optional[str] = None, **_):
        self.experiment_name = experiment_name
        if tracking_uri and tracking_uri not in ("databricks",):
            mlflow.set_tracking_uri(tracking_uri)

    def start(self):
        if ddist.get_rank() == 0:
            mlflow.set_experiment(self.experiment_name)
            if mlflow.active_run() is None:
                mlflow.start_run()

    def log_metrics(self, m: Dict[str, float], step: int):
        if ddist.get_rank() == 0:
            mlflow.log_metrics(m, step=step)


class Trainer:
    def __init__(self, model: nn.Module, optimizers=None, train_dataloader=None, eval_dataloader=None,
                 max_duration: str = "1ep", algorithms: Sequence[Algorithm] = (), loggers: Sequence[Any] = (),
                 device: Optional[str] = None, schedulers=None, **_):
        from ..engine.autograd_trainer import AutogradTrainer
        from ..config import OptimizerConfig
        self.info = ddist.init_distributed(device=device if device in ("cpu", "cuda") else None)
        self.native = False
        model = self._maybe_native(model, train_dataloader)
        smoothing = next((a.smoothing for a in algorithms if isinstance(a, LabelSmoothing)), 0.0)
        cut = next((a for a in algorithms if isinstance(a, CutMix)), None)
        oc = OptimizerConfig(name="adam", lr=1e-4, weight_decay=0.0)
        if optimizers is not None:
            g = optimizers.param_groups[0]
            name = type(optimizers).__name__.lower()
            oc = OptimizerConfig(name=name if name in ("sgd", "adam", "adamw") else "adam", lr=g["lr"],
                                 momentum=g.get("momentum", 0.9), weight_decay=g.get("weight_decay", 0.0),
                                 betas=tuple(g.get("betas", (0.9, 0.999))), eps=g.get("eps", 1e-8))
        self.tr = AutogradTrainer(model, self.info.device, oc, label_smoothing=smoothing,
                                  cutmix_alpha=cut.alpha if cut else 0.0)
        if cut and cut.num_classes:
            self.tr.num_classes = cut.num_classes
        self.train_dl, self.eval_dl = train_dataloader, eval_dataloader
        self.max_duration = max_duration
        self.loggers = list(loggers)
        self.state: Dict[str, Any] = {"epoch": 0, "batch": 0}
        self.history: List[Dict[str, float]] = []

    def _maybe_native(self, model, dl):
        import os
        from ..engine.native_module import native_module
        from ..engine.program import supports
        from ..models.wrappers import ComposerResNet50
        if (not EngineConfig.current().native_frontends or self.info.device.type != "cuda"
                or not isinstance(model, ComposerResNet50)):
            return model
        bs = getattr(dl, "batch_size", None)
        try:
            x0 = dl.dataset[0][0]
        except Exception:
            return model
        if not bs or not torch.is_tensor(x0) or x0.dim() != 3 or not supports(model.model):
            return model
        model.model = native_module(model.model, bs, tuple(x0.shape[1:]), self.info.device)
        self.native = True
        return model

    def fit(self):
        spe = len(self.train_dl)
        total = parse_duration(self.max_duration, spe, getattr(self.train_dl, "batch_size", 1) or 1)
        for lg in self.loggers:
            lg.start()
        step, epoch = 0, 0
        while step < total:
            n = 0
            for x, y in self.train_dl:
                if step >= total:
                    break
                self.tr.step(x, y)
                step += 1
                n += y.shape[0]
            epoch += 1
            loss, corr = self.tr.read_metrics()
            loss, corr, n = ddist.all_reduce_sum([loss, corr, float(n)])
            rec = {"train/loss": loss / max(1, n), "train/accuracy": corr / max(1, n)}
            if self.eval_dl is not None:
                el, ec, en = 0.0, 0.0, 0
                for x, y in self.eval_dl:
                    l, c = self.tr.eval_batch(x, y)
                    el, ec, en = el + l, ec + c, en + y.shape[0]
                el, ec, en = ddist.all_reduce_sum([el, ec, float(en)])
                rec.update({"metrics/eval/CrossEntropy": el / max(1, en), "metrics/eval/Accuracy": ec / max(1, en)})
            self.history.append(rec)
            for lg in self.loggers:
                lg.log_metrics(rec, step=epoch)
            self.state.update(epoch=epoch, batch=step)
        return self.history

    @property
    def model(self):
        return self.tr.model

    def close(self):
        if ddist.get_rank() == 0 and mlflow.active_run() is not None:
            mlflow.end_run()
