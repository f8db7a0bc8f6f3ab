"""Environment bootstrap: the ``%run ../setup/00_setup`` equivalent.

The reference's setup notebook (`setup/00_setup.py`) reads ``../local_config.yaml`` (`:7-23`),
creates the Unity-Catalog catalog/schema and four volumes with try/except-print (`:27-54`), sets
HF cache env plus ``CUDA_LAUNCH_BLOCKING=1`` / ``TORCH_DISTRIBUTED_DEBUG=DETAIL`` unconditionally
(`:58-67`), logs into Hugging Face from a secret (`:71-77`), captures host/token and sets the MLflow
experiment ``/Users/<user>/experiments/<notebook>`` (`:81-101`), and discovers workers/GPUs via
Spark (`:105-113`). ``setup()`` does the same on a standalone MI355X node:

* storage: volumes become directories under ``LocalConfig.volume_root/<catalog>/<schema>/``;
* env: HF cache vars; debug flags only when asked (``debug=1|2``, utils/debug.py) — launch
  blocking is never the default;
* secrets: token from ``$HF_TOKEN`` or ``~/.dbx_amd/secrets/<scope>/<key>``; login is recorded
  but nothing is fetched (the node is offline);
* MLflow: ``utils.mlflow_compat`` file store, same experiment path layout;
* GPUs: ``torch.cuda.device_count()`` (does not initialise HIP on this stack), workers from
  ``$DBX_NUM_WORKERS`` / ``LocalConfig.num_nodes``.
"""
from __future__ import annotations

import getpass
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional

from .config import LocalConfig, load_local_config
from .utils import debug as _debug

VOLUMES = ("cifar_cache", "tiny_imagenet_cache", "imagenet1k_cache", "coco_cache")


@dataclass
class SetupContext:
    config: LocalConfig
    volumes: Dict[str, str] = field(default_factory=dict)
    hf_home: str = ""
    hf_logged_in: bool = False
    username: str = ""
    experiment_path: str = ""
    experiment_id: Optional[str] = None
    num_workers: int = 1
    num_gpus_per_worker: int = 0
    errors: List[str] = field(default_factory=list)

    @property
    def world_size(self) -> int:
        return max(1, self.num_workers) * max(1, self.num_gpus_per_worker)


def provision_storage(lc: LocalConfig, names=VOLUMES, errors: Optional[List[str]] = None) -> Dict[str, str]:
    """CREATE CATALOG/SCHEMA/VOLUME IF NOT EXISTS -> mkdir -p; failures are reported, not raised
    (the reference prints and continues, `00_setup.py:27-54`)."""
    out = {}
    for n in names:
        path = lc.volume(n)
        try:
            os.makedirs(path, exist_ok=True)
            out[n] = path
        except OSError as e:
            msg = f"could not create volume {n} at {path}: {e}"
            if errors is not None:
                errors.append(msg)
    return out


def read_secret(scope: str, key: str) -> Optional[str]:
    """``dbutils.secrets.get(scope, key)`` stand-in: env ``DBX_SECRET_<SCOPE>_<KEY>`` or a file."""
    if not scope or not key:
        return None
    env = os.environ.get(f"DBX_SECRET_{scope}_{key}".upper().replace("-", "_"))
    if env:
        return env
    path = os.path.join(os.path.expanduser("~/.dbx_amd/secrets"), scope, key)
    if os.path.exists(path):
        with open(path) as f:
            return f.read().strip()
    return None


def hf_login(token: Optional[str]) -> bool:
    """Record the HF token for the hub client (offline: no network call is made)."""
    if not token:
        return False
    os.environ["HF_TOKEN"] = token
    return True


def discover_gpus() -> int:
    try:
        import torch
        return torch.cuda.device_count()
    except Exception:  # pragma: no cover - torch always importable here
        return 0


def setup(config_path: str = "../local_config.yaml", notebook_name: str = "notebook", debug: int = 0,
          hf_cache: Optional[str] = None, mlflow_root: Optional[str] = None) -> SetupContext:
    lc = load_local_config(config_path)
    ctx = SetupContext(config=lc)
    ctx.volumes = provision_storage(lc, errors=ctx.errors)
    # HF cache env (`00_setup.py:58-64`)
    ctx.hf_home = hf_cache or os.environ.get("DBX_HF_CACHE", os.path.join(lc.volume_root, "hf_cache"))
    os.makedirs(ctx.hf_home, exist_ok=True)
    os.environ["HF_HOME"] = ctx.hf_home
    os.environ["HUGGINGFACE_HUB_CACHE"] = ctx.hf_home
    os.environ["HF_HUB_DISABLE_SYMLINKS_WARNING"] = "True"
    os.environ.setdefault("HF_HUB_OFFLINE", "1")
    os.environ.setdefault("HF_DATASETS_OFFLINE", "1")
    if debug:
        os.environ.update(_debug.debug_env(debug))
    # secrets + HF login (`00_setup.py:71-77`)
    try:
        ctx.hf_logged_in = hf_login(os.environ.get("HF_TOKEN") or read_secret(lc.secret_scope, lc.secret_key))
    except Exception as e:  # pragma: no cover
        ctx.errors.append(f"could not log into huggingface: {e}")
    # MLflow experiment (`00_setup.py:81-101`)
    from .utils import mlflow_compat as mlflow
    if mlflow_root:
        mlflow.set_tracking_uri(mlflow_root)
    ctx.username = os.environ.get("DBX_USER") or getpass.getuser()
    ctx.experiment_path = f"/Users/{ctx.username}/experiments/{notebook_name}"
    ctx.experiment_id = mlflow.set_experiment(ctx.experiment_path)["experiment_id"]
    os.environ["MLFLOW_EXPERIMENT_NAME"] = ctx.experiment_path
    # workers / GPUs (`00_setup.py:105-113`)
    ctx.num_workers = int(os.environ.get("DBX_NUM_WORKERS", lc.num_nodes or 1))
    ctx.num_gpus_per_worker = discover_gpus()
    return ctx
