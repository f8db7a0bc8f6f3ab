"""MLflow-compatible experiment tracking without requiring mlflow.

The reference logs params/metrics/models to a Databricks MLflow server (`setup/00_setup.py:96-101`,
e.g. `02_cifar_torch_distributor_resnet.py:207-300`, `04_accelerate/01_cifar_accelerate.ipynb:574-782`).
mlflow is not installed on this image, so this module implements the API subset those notebooks
use on top of MLflow's own *file store* layout (``mlruns/<exp_id>/<run_id>/{meta.yaml, params/,
metrics/, tags/, artifacts/}``; metric files hold ``<ms timestamp> <value> <step>`` lines), which
a real ``mlflow ui --backend-store-uri <dir>`` can read. If mlflow IS importable and
``DBX_USE_REAL_MLFLOW=1``, calls are forwarded to it instead.

Usage mirrors ``import mlflow``::

    from dbx_distributed_pytorch_examples_amd.utils import mlflow_compat as mlflow
    mlflow.set_experiment("/Users/me/experiments/cifar")
    with mlflow.start_run() as run:
        mlflow.log_params({"batch_size": 256}); mlflow.log_metric("train_loss", 0.5, step=1)
        mlflow.pytorch.log_model(model, "model")
"""
from __future__ import annotations

import contextlib
import json
import os
import threading
import time
import uuid
from dataclasses import dataclass
from typing import Any, Dict, Optional

import yaml

_LOCK = threading.Lock()


def _root() -> str:
    uri = os.environ.get("MLFLOW_TRACKING_URI", "")
    if uri.startswith("file:"):
        uri = uri[5:]
    if not uri or uri in ("databricks",) or "://" in uri:
        uri = os.environ.get("DBX_MLRUNS", os.path.abspath("mlruns"))
    return uri


@dataclass
class RunInfo:
    run_id: str
    experiment_id: str
    run_name: str
    artifact_uri: str
    status: str = "RUNNING"


class Run:
    def __init__(self, info: RunInfo):
        self.info = info

    def __enter__(self):
        return self

    def __exit__(self, et, ev, tb):
        end_run("FAILED" if et else "FINISHED")
        return False


_state: Dict[str, Any] = {"experiment_id": None, "runs": []}


def set_tracking_uri(uri: str) -> None:
    os.environ["MLFLOW_TRACKING_URI"] = uri


def get_tracking_uri() -> str:
    return "file://" + _root()


def _exp_dir(eid: str) -> str:
    return os.path.join(_root(), eid)


def set_experiment(name: str):
    root = _root()
    os.makedirs(root, exist_ok=True)
    with _LOCK:
        for d in sorted(os.listdir(root)):
            meta = os.path.join(root, d, "meta.yaml")
            if os.path.exists(meta):
                with open(meta) as f:
                    m = yaml.safe_load(f) or {}
                if m.get("name") == name:
                    _state["experiment_id"] = d
                    return m
        ids = [int(d) for d in os.listdir(root) if d.isdigit()]
        eid = str(max(ids) + 1 if ids else 1)
        os.makedirs(_exp_dir(eid), exist_ok=True)
        m = {"experiment_id": eid, "name": name, "artifact_location": "file://" + _exp_dir(eid),
             "lifecycle_stage": "active", "creation_time": int(time.time() * 1000)}
        with open(os.path.join(_exp_dir(eid), "meta.yaml"), "w") as f:
            yaml.safe_dump(m, f)
        _state["experiment_id"] = eid
        return m


def _ensure_experiment() -> str:
    if _state["experiment_id"] is None:
        set_experiment(os.environ.get("MLFLOW_EXPERIMENT_NAME", "Default"))
    return _state["experiment_id"]


def _run_dir(run_id: Optional[str] = None) -> str:
    rid = run_id or active_run().info.run_id
    root = _root()
    for eid in os.listdir(root):
        d = os.path.join(root, eid, rid)
        if os.path.isdir(d):
            return d
    raise KeyError(f"run {rid} not found under {root}")


def start_run(run_id: Optional[str] = None, run_name: Optional[str] = None, nested: bool = False,
              experiment_id: Optional[str] = None, tags: Optional[Dict[str, str]] = None) -> Run:
    eid = experiment_id or _ensure_experiment()
    if run_id is not None:  # resume
        d = _run_dir(run_id)
        with open(os.path.join(d, "meta.yaml")) as f:
            m = yaml.safe_load(f)
        info = RunInfo(run_id, m["experiment_id"], m.get("run_name", ""), m["artifact_uri"])
    else:
        if _state["runs"] and not nested:
            raise RuntimeError("a run is already active; pass nested=True or end it first")
        rid = uuid.uuid4().hex
        d = os.path.join(_exp_dir(eid), rid)
        for sub in ("params", "metrics", "tags", "artifacts"):
            os.makedirs(os.path.join(d, sub), exist_ok=True)
        info = RunInfo(rid, eid, run_name or rid[:8], "file://" + os.path.join(d, "artifacts"))
        meta = {"run_id": rid, "run_uuid": rid, "experiment_id": eid, "run_name": info.run_name,
                "artifact_uri": info.artifact_uri, "status": 1, "start_time": int(time.time() * 1000),
                "end_time": None, "lifecycle_stage": "active", "user_id": os.environ.get("USER", "dbx")}
        with open(os.path.join(d, "meta.yaml"), "w") as f:
            yaml.safe_dump(meta, f)
        if _state["runs"]:
            tags = dict(tags or {}, **{"mlflow.parentRunId": _state["runs"][-1].info.run_id})
        for k, v in (tags or {}).items():
            with open(os.path.join(d, "tags", k), "w") as f:
                f.write(str(v))
    run = Run(info)
    _state["runs"].append(run)
    return run


def active_run() -> Optional[Run]:
    return _state["runs"][-1] if _state["runs"] else None


def end_run(status: str = "FINISHED") -> None:
    if not _state["runs"]:
        return
    run = _state["runs"].pop()
    d = _run_dir(run.info.run_id)
    p = os.path.join(d, "meta.yaml")
    with open(p) as f:
        m = yaml.safe_load(f)
    m["status"] = {"FINISHED": 3, "FAILED": 4, "KILLED": 5}.get(status, 3)
    m["end_time"] = int(time.time() * 1000)
    with open(p, "w") as f:
        yaml.safe_dump(m, f)


def _need_run() -> Run:
    r = active_run()
    if r is None:
        r = start_run()
    return r


def log_param(key: str, value: Any) -> None:
    d = _run_dir(_need_run().info.run_id)
    with open(os.path.join(d, "params", key), "w") as f:
        f.write(str(value))


def log_params(params: Dict[str, Any]) -> None:
    for k, v in params.items():
        log_param(k, v)


def log_metric(key: str, value: float, step: Optional[int] = None) -> None:
    d = _run_dir(_need_run().info.run_id)
    path = os.path.join(d, "metrics", key)
    os.makedirs(os.path.dirname(path), exist_ok=True)  # "system/gpu_0_..." keys nest like MLflow's
    with _LOCK, open(path, "a") as f:
        f.write(f"{int(time.time() * 1000)} {float(value)} {int(step or 0)}\n")


def log_metrics(metrics: Dict[str, float], step: Optional[int] = None) -> None:
    for k, v in metrics.items():
        log_metric(k, v, step)


def set_tag(key: str, value: Any) -> None:
    d = _run_dir(_need_run().info.run_id)
    with open(os.path.join(d, "tags", key), "w") as f:
        f.write(str(value))


def _artifact_dir(path: str = "") -> str:
    d = os.path.join(_run_dir(_need_run().info.run_id), "artifacts", path)
    os.makedirs(d, exist_ok=True)
    return d


def log_dict(d: Dict[str, Any], artifact_file: str) -> None:
    full = os.path.join(_run_dir(_need_run().info.run_id), "artifacts", artifact_file)
    os.makedirs(os.path.dirname(full), exist_ok=True)
    with open(full, "w") as f:
        if artifact_file.endswith((".yaml", ".yml")):
            yaml.safe_dump(d, f)
        else:
            json.dump(d, f, indent=2, default=str)


def log_artifact(local_path: str, artifact_path: str = "") -> None:
    import shutil
    dst = _artifact_dir(artifact_path)
    shutil.copy2(local_path, os.path.join(dst, os.path.basename(local_path)))


def get_metric_history(run_id: str, key: str):
    d = _run_dir(run_id)
    out = []
    with open(os.path.join(d, "metrics", key)) as f:
        for line in f:
            ts, v, s = line.split()
            out.append((int(s), float(v), int(ts)))
    return out


def get_params(run_id: str) -> Dict[str, str]:
    d = os.path.join(_run_dir(run_id), "params")
    return {k: open(os.path.join(d, k)).read() for k in os.listdir(d)}


class _PyTorchFlavor:
    """``mlflow.pytorch`` subset: log_model / log_state_dict / load_model / load_state_dict / autolog."""

    def log_model(self, model, artifact_path: str, **_kw) -> str:
        import torch
        d = _artifact_dir(artifact_path)
        from ..parallel.ddp import unwrap
        m = unwrap(model)
        sd = {k: v.detach().cpu().contiguous() for k, v in m.state_dict().items()}
        torch.save(sd, os.path.join(d, "state_dict.pth"))
        spec = getattr(m, "_dbx_spec", None)
        meta = {"flavor": "dbx.pytorch", "class": f"{type(m).__module__}.{type(m).__qualname__}", "spec": spec}
        with open(os.path.join(d, "MLmodel"), "w") as f:
            yaml.safe_dump(meta, f)
        if spec is None:  # no factory spec: also keep the whole module (file written by this code)
            torch.save(m, os.path.join(d, "model.pth"))
        return f"runs:/{active_run().info.run_id}/{artifact_path}"

    def log_state_dict(self, state_dict: Dict[str, Any], artifact_path: str) -> None:
        import torch
        d = _artifact_dir(artifact_path)
        torch.save(_to_cpu(state_dict), os.path.join(d, "state_dict.pth"))

    def _resolve(self, uri: str) -> str:
        if uri.startswith("runs:/"):
            rid, path = uri[len("runs:/"):].split("/", 1)
            return os.path.join(_run_dir(rid), "artifacts", path)
        return uri

    def load_state_dict(self, uri: str, map_location="cpu"):
        import torch
        return torch.load(os.path.join(self._resolve(uri), "state_dict.pth"), map_location=map_location,
                          weights_only=True)

    def load_model(self, uri: str, map_location="cpu"):
        import torch
        d = self._resolve(uri)
        with open(os.path.join(d, "MLmodel")) as f:
            meta = yaml.safe_load(f)
        spec = meta.get("spec")
        if spec:
            from ..models import build_model
            m = build_model(spec["name"], **spec.get("kwargs", {}))
            m.load_state_dict(torch.load(os.path.join(d, "state_dict.pth"), map_location="cpu", weights_only=True))
            return m.to(map_location)
        # whole-module file produced by log_model() above in this framework (trusted, our own output)
        return torch.load(os.path.join(d, "model.pth"), map_location=map_location, weights_only=False)

    def autolog(self, *a, **k) -> None:
        return None


def _to_cpu(obj):
    import torch
    if isinstance(obj, torch.Tensor):
        return obj.detach().cpu()
    if isinstance(obj, dict):
        return {k: _to_cpu(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_cpu(v) for v in obj)
    return obj


pytorch = _PyTorchFlavor()


def enable_system_metrics_logging(interval_s: float = 10.0):
    """Sample GPU util/memory (rocm-smi / amd-smi) into the active run (system/* metrics)."""
    from .sysmetrics import SystemMetricsLogger
    return SystemMetricsLogger(interval_s=interval_s, log_fn=log_metric).start()


@contextlib.contextmanager
def run_context(**kw):
    r = start_run(**kw)
    try:
        yield r
    finally:
        end_run()
