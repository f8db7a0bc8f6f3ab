"""HF-Accelerate-style API (`04_accelerate/01_cifar_accelerate.ipynb`) over our process group / DDP.

``Accelerator().prepare(model, optimizer, train_loader, eval_loader, scheduler)`` moves the model to
this rank's GPU (channels_last), wraps it in the flat-bucket DDP, re-shards the loaders with
``ShardSampler`` (their batches then arrive on the device) and returns them; ``backward(loss)`` runs autograd and finishes the bucket
all-reduces; ``gather`` / ``reduce`` are packed collectives; ``log`` forwards to the MLflow-compat
tracker (``log_with="mlflow"``). bf16 autocast is enabled by ``mixed_precision="bf16"``.

On a GPU, ``prepare`` puts a supported ResNet (the notebook's ``resnet50`` with a new ``fc``,
`04_accelerate/01_cifar_accelerate.ipynb:475-503`) on the native HIP kernels by default:
:func:`~dbx_distributed_pytorch_examples_amd.engine.native_module.native_module` compiles it for
the first training batch's shape (``DBX_ACCELERATE_NATIVE=0`` or ``mixed_precision="no"`` keep the
stock module). The Parameter objects do not change, so the optimizer the notebook built before
``prepare`` keeps stepping the live weights; the module all-reduces its own gradient per backward
segment, overlapped with the backward, so it is not wrapped in DDP. A model already wrapped by
``native_module`` is passed through as is. Any other model runs under ``torch.autocast(bf16)`` with
fp32 outputs when ``mixed_precision="bf16"`` (the default).
"""
from __future__ import annotations

import contextlib
import random
from typing import Any, List, Optional

import numpy as np
import torch
from torch.utils.data import DataLoader

from ..parallel import dist as ddist
from ..parallel.ddp import DistributedDataParallel, unwrap
from ..parallel.sampler import ShardSampler
from ..utils import mlflow_compat as mlflow


def set_seed(seed: int) -> None:
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)


class _PreparedOptimizer:
    def __init__(self, opt, acc):
        self.opt, self.acc = opt, acc

    def step(self, *a, **k):
        for m in self.acc._models:
            m.finish_gradient_sync()
        return self.opt.step(*a, **k)

    def zero_grad(self, set_to_none: bool = True):
        for m in self.acc._models:
            m.zero_grad()
        self.opt.zero_grad(set_to_none=False)

    def __getattr__(self, k):
        return getattr(self.opt, k)

    def state_dict(self):
        return self.opt.state_dict()

    def load_state_dict(self, sd):
        return self.opt.load_state_dict(sd)


class _DeviceLoader:
    """A prepared DataLoader: batches arrive on the accelerator's device (HF Accelerate's
    ``DataLoaderShard`` behaviour); every other attribute is the wrapped loader's."""

    def __init__(self, dl: DataLoader, device: torch.device):
        self.dl, self.device = dl, device

    def _move(self, b):
        if isinstance(b, torch.Tensor):
            return b.to(self.device, non_blocking=True)
        if isinstance(b, (list, tuple)):
            return type(b)(self._move(v) for v in b)
        if isinstance(b, dict):
            return {k: self._move(v) for k, v in b.items()}
        return b

    def __iter__(self):
        for b in self.dl:
            yield self._move(b)

    def __len__(self):
        return len(self.dl)

    def __getattr__(self, k):
        return getattr(self.dl, k)


class Accelerator:
    def __init__(self, log_with: Optional[str] = None, mixed_precision: str = "bf16", cpu: bool = False, **_):
        self.info = ddist.init_distributed(device="cpu" if cpu else None)
        self.device = self.info.device
        self.mixed_precision = mixed_precision
        self.log_with = log_with
        self._models: List[DistributedDataParallel] = []
        self._trackers = False

    @property
    def num_processes(self) -> int:
        return ddist.get_world_size()

    @property
    def process_index(self) -> int:
        return ddist.get_rank()

    @property
    def local_process_index(self) -> int:
        return self.info.local_rank

    @property
    def is_main_process(self) -> bool:
        return ddist.get_rank() == 0

    @property
    def is_local_main_process(self) -> bool:
        return self.info.local_rank == 0

    def print(self, *a, **k):
        if self.is_main_process:
            print(*a, **k)

    def _prep_one(self, obj):
        if isinstance(obj, torch.nn.Module):
            import os
            from ..engine.native_module import NativeResNet, native_module
            from ..engine.program import supports
            if isinstance(obj, NativeResNet):
                return obj  # on the device already; gradients all-reduced by its own backward
            if (self.device.type == "cuda" and self.mixed_precision == "bf16" and supports(obj)
                    and os.environ.get("DBX_ACCELERATE_NATIVE", "1") != "0"):
                return native_module(obj, None, None, self.device)  # compiled for the first batch
            m = obj.to(self.device)
            if self.device.type == "cuda":
                m = m.to(memory_format=torch.channels_last)
            d = DistributedDataParallel(m, autocast_dtype=torch.bfloat16 if self.mixed_precision == "bf16" else None)
            self._models.append(d)
            return d
        if isinstance(obj, torch.optim.Optimizer):
            return _PreparedOptimizer(obj, self)
        if isinstance(obj, DataLoader):
            dl = obj
            if ddist.get_world_size() > 1:
                shuffle = not isinstance(obj.sampler, torch.utils.data.SequentialSampler)
                dl = DataLoader(obj.dataset, batch_size=obj.batch_size, sampler=ShardSampler(obj.dataset, shuffle=shuffle),
                                num_workers=obj.num_workers, collate_fn=obj.collate_fn, pin_memory=obj.pin_memory,
                                drop_last=obj.drop_last)
            return _DeviceLoader(dl, self.device) if self.device.type != "cpu" else dl
        return obj  # schedulers etc.

    def prepare(self, *objs):
        out = tuple(self._prep_one(o) for o in objs)
        return out[0] if len(out) == 1 else out

    def autocast(self):
        enabled = self.device.type == "cuda" and self.mixed_precision == "bf16"
        return torch.autocast(self.device.type, dtype=torch.bfloat16, enabled=enabled)

    def backward(self, loss: torch.Tensor) -> None:
        loss.backward()
        for m in self._models:
            m.finish_gradient_sync()

    def gather(self, t: torch.Tensor) -> torch.Tensor:
        t = torch.as_tensor(t, device=self.device)
        if ddist.get_world_size() == 1:
            return t.reshape(1, *t.shape) if t.dim() == 0 else t
        import torch.distributed as dist
        parts = [torch.empty_like(t.reshape(-1) if t.dim() == 0 else t) for _ in range(ddist.get_world_size())]
        dist.all_gather(parts, t.reshape(-1) if t.dim() == 0 else t)
        return torch.cat(parts)

    def reduce(self, t: torch.Tensor, reduction: str = "sum") -> torch.Tensor:
        t = torch.as_tensor(t, device=self.device).clone()
        ddist.all_reduce_tensor_(t)
        if reduction == "mean":
            t /= ddist.get_world_size()
        return t

    def wait_for_everyone(self) -> None:
        ddist.barrier()

    def unwrap_model(self, model):
        return unwrap(model)

    def init_trackers(self, project_name: str, config: Optional[dict] = None, **_):
        if self.log_with == "mlflow" and self.is_main_process:
            mlflow.set_experiment(project_name)
            if mlflow.active_run() is None:
                mlflow.start_run()
            if config:
                mlflow.log_params(config)
            self._trackers = True

    def log(self, values: dict, step: Optional[int] = None) -> None:
        if self._trackers and self.is_main_process:
            mlflow.log_metrics({k: float(v) for k, v in values.items()}, step=step)

    def end_training(self) -> None:
        if self._trackers and self.is_main_process and mlflow.active_run() is not None:
            mlflow.end_run()
        self._trackers = False

    def save(self, obj, path: str) -> None:
        if self.is_main_process:
            torch.save(obj, path)

    @contextlib.contextmanager
    def no_sync(self, model):
        with model.no_sync():
            yield
