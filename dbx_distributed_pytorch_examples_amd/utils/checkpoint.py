"""Checkpoint layouts of the reference + real resume.

* ``checkpoint-{epoch}.pth.tar`` = ``{'model': state_dict, 'optimizer': state_dict}`` under a
  ``log_dir`` (`01_torch_distributor/01_basic_torch_distributor.py:109-124`, DDP variant saving the
  unwrapped module on rank 0, `:239-245`); extra keys are added for resume (``epoch``, ``step``,
  ``scheduler``, ``sampler_epoch``, ``rng``, ``trainer``) and ignored by reference readers.
* the Accelerate per-epoch dict ``{epoch, model_state_dict, optimizer_state_dict,
  scheduler_state_dict, test_accuracy}`` (`04_accelerate/01_cifar_accelerate.ipynb:711-725`);
* the Ray ``model.pt`` (unwrapped state dict in a directory, `05_ray/01_fashion_mnist_pytorch_ray.ipynb:203-219`).

State dicts are always written in torchvision layout (NCHW fp32, contiguous) even though the
native engine keeps conv weights as channels_last views of its flat master buffer. Every load
uses ``torch.load(..., weights_only=True)``.
"""
from __future__ import annotations

import glob
import os
import re
import time
from typing import Any, Dict, Optional

import torch

from ..parallel.ddp import unwrap

PYTORCH_DIR = os.environ.get("DBX_PYTORCH_DIR", os.path.expanduser("~/.dbx_amd/ml/pytorch"))


def create_log_dir(base: Optional[str] = None) -> str:
    """``/dbfs/ml/pytorch/<time()>`` of the reference -> ``$DBX_PYTORCH_DIR/<time()>``."""
    d = os.path.join(base or PYTORCH_DIR, str(time.time()))
    os.makedirs(d, exist_ok=True)
    return d


def clean_state_dict(sd: Dict[str, Any]) -> Dict[str, Any]:
    out = {}
    for k, v in sd.items():
        out[k] = v.detach().cpu().contiguous() if isinstance(v, torch.Tensor) else v
    return out


def model_state(model) -> Dict[str, Any]:
    return clean_state_dict(unwrap(model).state_dict())


def _rng_state() -> Dict[str, Any]:
    st = {"cpu": torch.get_rng_state()}
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        st["cuda"] = torch.cuda.get_rng_state()
    return st


def save_checkpoint(log_dir: str, model, optimizer=None, epoch: int = 0, **extra) -> str:
    os.makedirs(log_dir, exist_ok=True)
    path = os.path.join(log_dir, f"checkpoint-{epoch}.pth.tar")
    state = {"model": model_state(model)}
    if optimizer is not None:
        state["optimizer"] = clean_state_dict(optimizer.state_dict()) if hasattr(optimizer, "state_dict") else optimizer
    state["epoch"] = epoch
    state["rng"] = _rng_state()
    state.update(extra)
    tmp = path + ".tmp"
    torch.save(state, tmp)
    os.replace(tmp, path)  # atomic: a crash mid-write never leaves a truncated checkpoint
    return path


def load_checkpoint(log_dir: str, epoch: Optional[int] = None, map_location="cpu") -> Dict[str, Any]:
    path = os.path.join(log_dir, f"checkpoint-{epoch}.pth.tar") if epoch is not None else latest_checkpoint(log_dir)
    if path is None or not os.path.exists(path):
        raise FileNotFoundError(f"no checkpoint in {log_dir} (epoch={epoch})")
    return torch.load(path, map_location=map_location, weights_only=True)


def latest_checkpoint(log_dir: str) -> Optional[str]:
    best, best_e = None, -1
    for p in glob.glob(os.path.join(log_dir, "checkpoint-*.pth.tar")):
        m = re.search(r"checkpoint-(\d+)\.pth\.tar$", p)
        if m and int(m.group(1)) > best_e:
            best, best_e = p, int(m.group(1))
    return best


def restore_rng(state: Dict[str, Any]) -> None:
    r = state.get("rng")
    if not r:
        return
    torch.set_rng_state(r["cpu"])
    if "cuda" in r and torch.cuda.is_available():
        torch.cuda.set_rng_state(r["cuda"])


def accelerate_checkpoint(epoch: int, model, optimizer=None, scheduler=None, test_accuracy: float = 0.0) -> Dict:
    """The Accelerate notebook's per-epoch dict (logged with mlflow.pytorch.log_state_dict)."""
    return {
        "epoch": epoch,
        "model_state_dict": model_state(model),
        "optimizer_state_dict": clean_state_dict(optimizer.state_dict()) if optimizer is not None else None,
        "scheduler_state_dict": scheduler.state_dict() if scheduler is not None else None,
        "test_accuracy": float(test_accuracy),
    }


def save_ray_checkpoint(directory: str, model) -> str:
    os.makedirs(directory, exist_ok=True)
    p = os.path.join(directory, "model.pt")
    torch.save(model_state(model), p)
    return p


def load_ray_checkpoint(directory: str, map_location="cpu") -> Dict[str, Any]:
    return torch.load(os.path.join(directory, "model.pt"), map_location=map_location, weights_only=True)
