"""Ray-Train-style API (`05_ray/01_fashion_mnist_pytorch_ray.ipynb`, `05_ray/02_cifar_resnet_pytorch_ray.ipynb`).

``TorchTrainer(train_func, scaling_config=ScalingConfig(num_workers=N, use_gpu=True),
run_config=RunConfig(storage_path, name)).fit()`` runs ``train_func`` on N ranks through the native
launcher (no Ray cluster: ``setup_ray_cluster`` / ``shutdown_ray_cluster`` are no-op shims for
notebook parity). Inside workers: ``report(metrics, checkpoint=Checkpoint.from_directory(d))``,
``get_context().get_world_rank()``, ``prepare_model`` (device + flat-bucket DDP) and
``prepare_data_loader`` (ShardSampler + device moves). ``fit()`` returns a ``Result`` with the last
metrics, the last checkpoint (copied under ``storage_path/name``), the path and any error.
"""
from __future__ import annotations

import json
import os
import shutil
import tempfile
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional

import torch
from torch.utils.data import DataLoader

from ..launch import Launcher, LaunchError
from ..parallel import dist as ddist
from ..parallel.ddp import DistributedDataParallel
from ..parallel.sampler import ShardSampler
from ..engine_config import EngineConfig


@dataclass
class ScalingConfig:
    num_workers: int = 1
    use_gpu: bool = True
    resources_per_worker: Optional[dict] = None


@dataclass
class RunConfig:
    storage_path: str = os.path.expanduser("~/.dbx_amd/ray_results")
    name: str = "dbx_run"
    failure_config: Optional[Any] = None


@dataclass
class FailureConfig:
    max_failures: int = 0


class Checkpoint:
    def __init__(self, path: str):
        self.path = path

    @classmethod
    def from_directory(cls, path: str) -> "Checkpoint":
        return cls(path)

    def as_directory(self):
        import contextlib

        @contextlib.contextmanager
        def _cm():
            yield self.path
        return _cm()

    def to_directory(self, path: Optional[str] = None) -> str:
        path = path or tempfile.mkdtemp()
        shutil.copytree(self.path, path, dirs_exist_ok=True)
        return path


@dataclass
class Result:
    metrics: Dict[str, Any] = field(default_factory=dict)
    checkpoint: Optional[Checkpoint] = None
    path: str = ""
    error: Optional[BaseException] = None
    metrics_history: List[Dict[str, Any]] = field(default_factory=list)


class _Context:
    def get_world_rank(self):
        return ddist.get_rank()

    def get_world_size(self):
        return ddist.get_world_size()

    def get_local_rank(self):
        return int(os.environ.get("LOCAL_RANK", "0"))

    def get_trial_dir(self):
        return os.environ.get("DBX_RAY_TRIAL_DIR", "")


def get_context() -> _Context:
    return _Context()


def report(metrics: Dict[str, Any], checkpoint: Optional[Checkpoint] = None) -> None:
    """Rank 0 appends metrics (and copies the checkpoint dir) into the trial directory."""
    trial = os.environ.get("DBX_RAY_TRIAL_DIR")
    if not trial or ddist.get_rank() != 0:
        return
    os.makedirs(trial, exist_ok=True)
    with open(os.path.join(trial, "result.json"), "a") as f:
        f.write(json.dumps({k: (float(v) if isinstance(v, (int, float)) else str(v)) for k, v in metrics.items()}) + "\n")
    if checkpoint is not None:
        n = len([d for d in os.listdir(trial) if d.startswith("checkpoint_")])
        shutil.copytree(checkpoint.path, os.path.join(trial, f"checkpoint_{n:06d}"), dirs_exist_ok=True)


def prepare_model(model: torch.nn.Module, native_batch: Optional[int] = None, native_hw=None,
                  **ddp_kw) -> torch.nn.Module:
    """``ray.train.torch.prepare_model`` (`05_ray/02_cifar_resnet_pytorch_ray.ipynb:280`). On a GPU a
    supported ResNet runs the worker's own loop on the native HIP program by default
    (``engine.native_module``, compiled for the first training batch's shape unless ``native_batch``
    / ``native_hw`` fix it; its backward averages the gradients per segment, overlapped with the
    backward; ``native_batch=0`` or the engine field ``native_frontends=0`` opt out). Otherwise the model is moved to
    the device and wrapped in the flat-bucket DDP at world > 1."""
    info = ddist.init_distributed(device="cpu" if os.environ.get("DBX_FORCE_CPU") == "1" else None)
    if (native_batch != 0 and info.device.type == "cuda" and EngineConfig.current().native_frontends):
        from ..engine.native_module import native_module
        from ..engine.program import supports
        if supports(model):
            return native_module(model, native_batch or None, tuple(native_hw) if native_hw else None,
                                 info.device)
    model = model.to(info.device)
    if info.device.type == "cuda":
        model = model.to(memory_format=torch.channels_last)
    return DistributedDataParallel(model, **ddp_kw) if ddist.get_world_size() > 1 else model


class _DeviceLoader:
    def __init__(self, dl: DataLoader, device):
        self.dl, self.device = dl, device
        self.sampler = dl.sampler

    def __iter__(self):
        for x, y in self.dl:
            yield x.to(self.device, non_blocking=True), y.to(self.device, non_blocking=True)

    def __len__(self):
        return len(self.dl)


def prepare_data_loader(dl: DataLoader, move_to_device: bool = True):
    info = ddist.init_distributed(device="cpu" if os.environ.get("DBX_FORCE_CPU") == "1" else None)
    if ddist.get_world_size() > 1:
        shuffle = not isinstance(dl.sampler, torch.utils.data.SequentialSampler)
        dl = DataLoader(dl.dataset, batch_size=dl.batch_size, sampler=ShardSampler(dl.dataset, shuffle=shuffle),
                        num_workers=dl.num_workers, collate_fn=dl.collate_fn, pin_memory=dl.pin_memory)
    return _DeviceLoader(dl, info.device) if move_to_device else dl


def setup_ray_cluster(*_a, **_k):
    """No Ray on this stack: ranks are native processes (kept for notebook parity)."""
    return "local"


def shutdown_ray_cluster():
    return None


def _worker_entry(fn, config):
    ddist.init_distributed(device="cpu" if os.environ.get("DBX_FORCE_CPU") == "1" else None)
    try:
        return fn(config) if config is not None else fn()
    finally:
        ddist.destroy()


class TorchTrainer:
    def __init__(self, train_loop_per_worker: Callable, train_loop_config: Optional[dict] = None,
                 scaling_config: Optional[ScalingConfig] = None, run_config: Optional[RunConfig] = None, **_):
        self.fn = train_loop_per_worker
        self.cfg = train_loop_config
        self.sc = scaling_config or ScalingConfig()
        self.rc = run_config or RunConfig()

    def fit(self) -> Result:
        trial = os.path.join(self.rc.storage_path, self.rc.name)
        os.makedirs(trial, exist_ok=True)
        retries = self.rc.failure_config.max_failures if self.rc.failure_config else 0
        L = Launcher(self.sc.num_workers, use_gpu=self.sc.use_gpu, max_restarts=retries,
                     env={"DBX_RAY_TRIAL_DIR": trial, **({} if self.sc.use_gpu else {"DBX_FORCE_CPU": "1"})})
        res = Result(path=trial)
        try:
            L.run(_worker_entry, self.fn, self.cfg)
        except LaunchError as e:
            res.error = e
        rj = os.path.join(trial, "result.json")
        if os.path.exists(rj):
            with open(rj) as f:
                res.metrics_history = [json.loads(l) for l in f if l.strip()]
            res.metrics = res.metrics_history[-1] if res.metrics_history else {}
        cks = sorted(d for d in os.listdir(trial) if d.startswith("checkpoint_"))
        if cks:
            res.checkpoint = Checkpoint(os.path.join(trial, cks[-1]))
        return res
