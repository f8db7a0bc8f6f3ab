"""Typed configuration: one dataclass tree, loadable from YAML/JSON/dicts with ``a.b=c`` overrides.

Replaces the reference's scattered configuration:

* ``local_config.yaml`` keys (`/root/reference/UPDATE_local_config.yaml:1-7`, read by
  `setup/00_setup.py:7-23`): ``catalog, schema, num_nodes, secret_scope, secret_key,
  cifar_cache, tiny_imagenet_cache, imagenet1k_cache, coco_cache`` -> :class:`LocalConfig`
  (Unity-Catalog volumes become local directories under ``volume_root``);
* per-file hyper-parameter constants (§2.3) -> :class:`TrainConfig`;
* DeepSpeed JSON dicts (`02_deepspeed/deepspeed_config.py`) -> :func:`from_deepspeed`;
* Composer duration strings ``"2ep"`` / ``"100ba"`` (`03_composer/01_cifar_composer_resnet.ipynb:287`)
  -> :func:`parse_duration`.
"""
from __future__ import annotations

import copy
import dataclasses
import json
import os
import re
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence, Tuple, Union

import yaml


@dataclass
class LocalConfig:
    """The reference's local_config.yaml (template `UPDATE_local_config.yaml:1-7` + `coco_cache`)."""
    catalog: str = ""
    schema: str = ""
    num_nodes: int = 1
    secret_scope: str = ""
    secret_key: str = ""
    cifar_cache: str = "cifar"
    tiny_imagenet_cache: str = "tiny_imagenet"
    imagenet1k_cache: str = "imagenet_1k"
    coco_cache: str = "ms_coco"
    volume_root: str = os.environ.get("DBX_VOLUME_ROOT", os.path.expanduser("~/.dbx_amd/volumes"))

    def volume(self, name: str) -> str:
        """Map a UC volume path (``/Volumes/<cat>/<schema>/<vol>``) or bare name to a local dir."""
        v = getattr(self, name, name)
        if v.startswith("/Volumes/"):
            v = v[len("/Volumes/"):]
        path = v if os.path.isabs(v) else os.path.join(self.volume_root, self.catalog or "main",
                                                        self.schema or "default", v)
        return path


@dataclass
class OptimizerConfig:
    name: str = "sgd"                  # sgd | adam | adamw | lars
    lr: float = 0.1
    momentum: float = 0.9
    nesterov: bool = False
    weight_decay: float = 5e-5
    betas: Tuple[float, float] = (0.9, 0.999)
    eps: float = 1e-8
    grad_clip: float = 0.0
    trust_coefficient: float = 0.001   # LARS eta


@dataclass
class SchedulerConfig:
    name: str = "none"                 # none | cosine | warmup_linear | warmup_cosine | step | warmup_lr
    warmup_steps: int = 0
    warmup_min_lr: float = 0.0
    warmup_type: str = "log"           # DeepSpeed WarmupLR: "log" (its default) | "linear"
    total_steps: int = 0
    t_max_epochs: int = 0              # CosineAnnealingLR(T_max=epochs), per-epoch stepping
    step_size: int = 30
    gamma: float = 0.1


@dataclass
class ZeroConfig:
    stage: int = 0                     # 0 = plain DDP, 1 = sharded optimizer state, 2 = + sharded grads, 3 = + sharded params
    reduce_bucket_size: int = 500_000_000
    allgather_bucket_size: int = 500_000_000
    overlap_comm: bool = True
    contiguous_gradients: bool = True
    reduce_scatter: bool = True
    offload_optimizer: bool = False    # fp32 master shard + moments in pinned host memory, CPU step (stage 3 path)
    offload_param: bool = False        # + no persistent device parameter shard
    allgather_partitions: bool = True
    sub_group_size: int = 1_000_000_000
    # stage 3 (parallel/fsdp.py): parameters smaller than the persistence threshold stay replicated
    # (never gathered / released); the prefetch size bounds how many parameter elements the next units'
    # all-gathers may run ahead of the forward; live / reuse distance are recorded (DeepSpeed
    # memory-pressure knobs with no effect at ResNet sizes on 288 GB HBM)
    stage3_prefetch_bucket_size: int = 50_000_000
    stage3_param_persistence_threshold: int = 100_000
    stage3_max_live_parameters: int = 1_000_000_000
    stage3_max_reuse_distance: int = 1_000_000_000
    stage3_gather_16bit_weights_on_model_save: bool = False


@dataclass
class DataConfig:
    dataset: str = "synthetic"         # synthetic | cifar10 | mnist | fashion_mnist | tiny_imagenet | imagenet | mds | folder | hf
    root: str = ""
    image_size: int = 224
    num_classes: int = 1000
    train_samples: int = 0             # synthetic: samples per epoch (0 = 50 batches)
    augment: bool = True
    num_workers: int = 4
    mds_remote: str = ""
    mds_local: str = ""
    shuffle: bool = True
    label_smoothing: float = 0.0
    cutmix_alpha: float = 0.0


@dataclass
class TrainConfig:
    model: str = "resnet50"
    num_classes: int = 1000
    batch_size: int = 256              # per GPU (micro batch)
    grad_accum: int = 1
    epochs: int = 1
    max_steps: int = 0                 # 0 = full epochs
    duration: str = ""                 # composer style: "2ep" / "100ba"
    seed: int = 42
    precision: str = "bf16"
    engine: str = "auto"               # auto | native | autograd
    graphs: bool = True
    bucket_cap_mb: float = 64.0
    allreduce_dtype: str = "fp32"
    log_every: int = 100
    eval_every: int = 1
    patience: int = 0                  # early stopping (02_tiny_imagenet_deepspeed_resnet.py:289-297)
    checkpoint_dir: str = ""
    checkpoint_every: int = 1
    resume: str = ""                   # path or "latest"
    experiment: str = "dbx_amd"
    run_name: str = ""
    model_name: str = "model"          # MLflow model artifact name (the notebooks' per-file names)
    wall_clock_breakdown: bool = False # DeepSpeed wall_clock_breakdown: per-phase timers (utils/profiling.py)
    tensorboard_dir: str = ""          # DeepSpeed tensorboard.output_path when enabled (recorded; MLflow is the sink)
    optim: OptimizerConfig = field(default_factory=OptimizerConfig)
    sched: SchedulerConfig = field(default_factory=SchedulerConfig)
    zero: ZeroConfig = field(default_factory=ZeroConfig)
    data: DataConfig = field(default_factory=DataConfig)
    local: LocalConfig = field(default_factory=LocalConfig)


# ----------------------------------------------------------------------------------------
def _coerce(cur: Any, val: Any) -> Any:
    if isinstance(cur, bool):
        if isinstance(val, str):
            return val.lower() in ("1", "true", "yes", "on")
        return bool(val)
    if isinstance(cur, int) and not isinstance(cur, bool):
        return int(float(val)) if isinstance(val, str) else int(val)
    if isinstance(cur, float):
        return float(val)
    if isinstance(cur, tuple):
        if isinstance(val, str):
            val = [float(x) for x in val.strip("()[]").split(",")]
        return tuple(type(c)(v) for c, v in zip(cur, val))
    return val


def update_dataclass(obj: Any, d: Dict[str, Any], strict: bool = True) -> Any:
    for k, v in d.items():
        if not hasattr(obj, k):
            if strict:
                raise KeyError(f"unknown config key {k!r} for {type(obj).__name__}")
            continue
        cur = getattr(obj, k)
        if dataclasses.is_dataclass(cur) and isinstance(v, dict):
            update_dataclass(cur, v, strict)
        else:
            setattr(obj, k, _coerce(cur, v) if cur is not None else v)
    return obj


def apply_overrides(cfg: Any, overrides: Sequence[str]) -> Any:
    """CLI overrides ``a.b=c`` (values parsed as YAML scalars)."""
    for ov in overrides:
        if "=" not in ov:
            raise ValueError(f"override {ov!r} is not key=value")
        key, val = ov.split("=", 1)
        parts = key.split(".")
        obj = cfg
        for p in parts[:-1]:
            obj = getattr(obj, p)
        if not hasattr(obj, parts[-1]):
            raise KeyError(f"unknown config key {key!r}")
        cur = getattr(obj, parts[-1])
        parsed = yaml.safe_load(val)
        setattr(obj, parts[-1], _coerce(cur, parsed) if cur is not None else parsed)
    return cfg


def load_config(path: Optional[str] = None, overrides: Sequence[str] = (), base: Optional[TrainConfig] = None
                ) -> TrainConfig:
    cfg = copy.deepcopy(base) if base is not None else TrainConfig()
    if path:
        with open(path) as f:
            d = json.load(f) if path.endswith(".json") else yaml.safe_load(f)
        d = d or {}
        if "train_micro_batch_size_per_gpu" in d or "zero_optimization" in d:
            cfg = from_deepspeed(d, cfg)
        elif set(d) & set(f.name for f in dataclasses.fields(LocalConfig)) and not set(d) & {"model", "optim"}:
            update_dataclass(cfg.local, d, strict=False)
        else:
            update_dataclass(cfg, d)
    return apply_overrides(cfg, overrides)


def load_local_config(path: str = "../local_config.yaml") -> LocalConfig:
    """``setup/00_setup.py:9-23`` equivalent; missing file -> defaults."""
    lc = LocalConfig()
    if os.path.exists(path):
        with open(path) as f:
            update_dataclass(lc, yaml.safe_load(f) or {}, strict=False)
    return lc


def to_dict(cfg: Any) -> Dict[str, Any]:
    return dataclasses.asdict(cfg)


# ----------------------------------------------------------------------------------------
_DUR = re.compile(r"^\s*(\d+(?:\.\d+)?)\s*(ep|ba|sp)\s*$")


def parse_duration(s: Union[str, int], steps_per_epoch: int, batch_size: int = 1) -> int:
    """Composer duration -> number of optimizer steps: ``"2ep"``, ``"100ba"``, ``"5000sp"`` (samples)."""
    if isinstance(s, int):
        return s * steps_per_epoch
    m = _DUR.match(s)
    if not m:
        raise ValueError(f"bad duration {s!r} (expected e.g. '2ep', '100ba', '5000sp')")
    v, unit = float(m.group(1)), m.group(2)
    if unit == "ep":
        return int(round(v * steps_per_epoch))
    if unit == "ba":
        return int(v)
    return int(v) // max(1, batch_size)


def _ds_auto(v: Any) -> bool:
    return isinstance(v, str) and v.strip().lower() == "auto"


def _ds_bool(v: Any, default: bool = False) -> bool:
    """DeepSpeed booleans: JSON true/false, or the strings "true"/"false" the reference writes
    (`deepspeed_config.py:19-21` has ``"enabled": "true"``); "auto" = ``default``."""
    if v is None or _ds_auto(v):
        return default
    if isinstance(v, str):
        s = v.strip().lower()
        if s in ("true", "1", "yes", "on"):
            return True
        if s in ("false", "0", "no", "off", ""):
            return False
        raise ValueError(f"not a DeepSpeed boolean: {v!r}")
    return bool(v)


def _ds_num(v: Any, auto: Union[int, float]) -> Union[int, float]:
    """A DeepSpeed number: int, float, numeric string ("5e8"), or "auto" -> ``auto``."""
    if _ds_auto(v):
        return auto
    return float(v) if isinstance(v, str) else v


# DeepSpeed's own optimizer defaults: a key the dict omits takes these, never a TrainConfig default.
# DeepSpeed builds "Adam" / "AdamW" as its FusedAdam (adam_w_mode for "AdamW"), whose weight_decay
# defaults to 0.0 -- not torch.optim.AdamW's 0.01 (the reference dicts omit the key,
# `02_deepspeed/deepspeed_config.py:22-32`, so their runs do not decay); SGD: torch's defaults.
_DS_OPT_DEFAULTS = {"adamw": {"weight_decay": 0.0}, "adam": {"weight_decay": 0.0},
                    "sgd": {"weight_decay": 0.0, "momentum": 0.0}}


def from_deepspeed(ds: Dict[str, Any], base: Optional[TrainConfig] = None, world_size: Optional[int] = None,
                   model_numel: Optional[int] = None) -> TrainConfig:
    """Map a DeepSpeed config dict (the schema `02_deepspeed/deepspeed_config.py:5-105` uses) onto a
    :class:`TrainConfig`. The reference dicts load verbatim:

    * ``"auto"`` values are resolved the way DeepSpeed's integration resolves them, with the model
      in place of a transformer's hidden size: ``train_batch_size`` = micro x accumulation x world,
      ``reduce_bucket_size`` / ``allgather_bucket_size`` = the whole gradient (``model_numel``; one
      bucket -- ResNet gradients are <= 102 MB), ``stage3_prefetch_bucket_size`` = 0.9 x that,
      ``stage3_param_persistence_threshold`` = DeepSpeed's default 1e5;
    * string booleans (``"true"`` / ``"false"``) are parsed, not truth-tested;
    * an explicit ``train_batch_size`` is checked against micro x accumulation x world (as DeepSpeed
      does) or, without a micro batch, defines it;
    * optimizer keys the dict omits take DeepSpeed's optimizer defaults (FusedAdam: weight decay 0.0
      for "Adam" and "AdamW"), not the TrainConfig's;
    * WarmupLR keeps its ``warmup_type`` ("log" when absent, DeepSpeed's default).
    """
    cfg = copy.deepcopy(base) if base is not None else TrainConfig()
    if world_size is None:
        world_size = int(os.environ.get("WORLD_SIZE", "1"))
    ga = ds.get("gradient_accumulation_steps", 1)
    ga = 1 if _ds_auto(ga) else int(float(ga))
    cfg.grad_accum = ga
    mb = ds.get("train_micro_batch_size_per_gpu")
    if mb is not None and not _ds_auto(mb):
        cfg.batch_size = int(float(mb))
    tbs = ds.get("train_batch_size")
    if tbs is not None and not _ds_auto(tbs):
        tbs = int(float(tbs))
        if mb is None or _ds_auto(mb):
            if tbs % (ga * world_size):
                raise ValueError(f"train_batch_size {tbs} is not divisible by accumulation {ga} x world {world_size}")
            cfg.batch_size = tbs // (ga * world_size)
        elif tbs != cfg.batch_size * ga * world_size:
            raise ValueError(f"train_batch_size {tbs} != micro batch {cfg.batch_size} x accumulation {ga} x "
                             f"world {world_size}")
    if "gradient_clipping" in ds and not _ds_auto(ds["gradient_clipping"]):
        cfg.optim.grad_clip = float(ds["gradient_clipping"])
    if _ds_bool(ds.get("bf16", {}).get("enabled")) or _ds_bool(ds.get("fp16", {}).get("enabled")):
        cfg.precision = "bf16"  # fp16 dicts too: the MI355X path computes in bf16 (no loss scaling needed)
    elif "bf16" in ds or "fp16" in ds:
        cfg.precision = "fp32"
    if "steps_per_print" in ds:
        cfg.log_every = int(float(ds["steps_per_print"]))
    if "wall_clock_breakdown" in ds:
        cfg.wall_clock_breakdown = _ds_bool(ds["wall_clock_breakdown"])
    tb = ds.get("tensorboard") or {}
    if _ds_bool(tb.get("enabled")):
        cfg.tensorboard_dir = str(tb.get("output_path", ""))
    opt = ds.get("optimizer")
    if opt:
        t = opt.get("type", "AdamW").lower()
        if t not in ("adamw", "adam", "sgd", "lars"):
            raise ValueError(f"unsupported DeepSpeed optimizer type {opt.get('type')!r}")
        cfg.optim.name = t
        p = dict(_DS_OPT_DEFAULTS.get(t, {}))
        p.update({"betas": (0.9, 0.999), "eps": 1e-8} if t in ("adamw", "adam") else {})
        p.update({k: v for k, v in opt.get("params", {}).items() if not _ds_auto(v)})
        if "lr" in p:
            cfg.optim.lr = float(p["lr"])
        if "betas" in p:
            cfg.optim.betas = tuple(float(b) for b in p["betas"])
        if "eps" in p:
            cfg.optim.eps = float(p["eps"])
        if "weight_decay" in p:
            cfg.optim.weight_decay = float(p["weight_decay"])
        if "momentum" in p:
            cfg.optim.momentum = float(p["momentum"])
    sch = ds.get("scheduler")
    if sch:
        t = sch.get("type", "")
        p = {k: v for k, v in sch.get("params", {}).items() if not _ds_auto(v)}
        if t == "WarmupLR":
            cfg.sched.name = "warmup_lr"
            cfg.sched.warmup_steps = int(float(p.get("warmup_num_steps", 1000)))
            cfg.sched.warmup_min_lr = float(p.get("warmup_min_lr", 0.0))
            cfg.sched.warmup_type = str(p.get("warmup_type", "log"))
            if cfg.sched.warmup_type not in ("log", "linear"):
                raise ValueError(f"WarmupLR warmup_type must be 'log' or 'linear', got {cfg.sched.warmup_type!r}")
            if "warmup_max_lr" in p:
                cfg.optim.lr = float(p["warmup_max_lr"])
        elif t in ("WarmupDecayLR", "WarmupCosineLR"):
            cfg.sched.name = "warmup_linear" if t == "WarmupDecayLR" else "warmup_cosine"
            cfg.sched.warmup_steps = int(float(p.get("warmup_num_steps", 0)))
            cfg.sched.warmup_type = str(p.get("warmup_type", "log"))
            cfg.sched.total_steps = int(float(p.get("total_num_steps", 0)))
        elif t:
            raise ValueError(f"unsupported DeepSpeed scheduler type {t!r}")
    z = ds.get("zero_optimization")
    if z is not None:
        zc = cfg.zero
        zc.stage = int(float(z.get("stage", 0)))
        whole = int(model_numel) if model_numel else zc.reduce_bucket_size
        for k in ("reduce_bucket_size", "allgather_bucket_size", "sub_group_size", "stage3_max_live_parameters",
                  "stage3_max_reuse_distance"):
            if k in z:
                setattr(zc, k, int(_ds_num(z[k], whole if "bucket" in k else getattr(zc, k))))
        if "stage3_prefetch_bucket_size" in z:
            zc.stage3_prefetch_bucket_size = int(_ds_num(z["stage3_prefetch_bucket_size"], 0.9 * whole))
        if "stage3_param_persistence_threshold" in z:
            zc.stage3_param_persistence_threshold = int(_ds_num(z["stage3_param_persistence_threshold"], 100_000))
        for k in ("overlap_comm", "contiguous_gradients", "reduce_scatter", "allgather_partitions",
                  "stage3_gather_16bit_weights_on_model_save"):
            if k in z:
                setattr(zc, k, _ds_bool(z[k], getattr(zc, k)))

        def _dev(key):
            d = z.get(key) or {}
            return str(d.get("device", "none")).lower() not in ("none", "") if isinstance(d, dict) else _ds_bool(d)
        zc.offload_optimizer = _dev("offload_optimizer") or _ds_bool(z.get("cpu_offload"))
        zc.offload_param = _dev("offload_param")
    cfg.deepspeed_applied = True  # train() then skips the launcher's DBX_DEEPSPEED_CONFIG env copy
    return cfg
