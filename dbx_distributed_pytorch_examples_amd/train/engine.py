"""``train()`` / ``evaluate()``: the one training loop behind every frontend.

The reference has one copy-pasted loop per notebook with the
same shape: per-epoch train loss/accuracy, rank-0 MLflow logging, rank-0 evaluation, model
logging, checkpoints. This module implements that loop once:

* engine selection: the graph-captured native ResNet program (``engine.native_trainer``) when
  the model is a supported ResNet on a GPU, else the autograd engine (any module, CPU or GPU);
* data: any map-style dataset (sharded by ``ShardSampler``) or an MDS ``StreamingDataset``;
  native engine batches go through ``data.loader.NativeImageLoader`` (pinned uint8 + GPU aug);
* metrics: ONE packed all-reduce per epoch (loss sum, correct, count), logged on rank 0 with the
  reference's names (``train_loss``, ``train_accuracy``, ``val_loss``, ``val_accuracy``,
  ``learning_rate``); no per-step ``.item()`` host syncs (the reference does two per step);
* evaluation: sharded over ranks and reduced (the reference evaluates on rank 0 only, or on
  every rank redundantly in 03a), deterministic transforms (no train-time augmentation on val);
* checkpoints: ``checkpoint-{epoch}.pth.tar`` (rank 0) with full resume state; ``resume="latest"``
  continues from the newest one (used by launcher restarts);
* early stopping on validation loss with ``patience`` (`02_deepspeed/02_tiny_imagenet_deepspeed_resnet.py:289-297`,
  made rank-consistent: the stop decision is broadcast, the reference only breaks on rank 0);
* fault tolerance: heartbeat + injection points every step; non-finite loss aborts all ranks.
"""
from __future__ import annotations

import json
import math
import os
import time
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Tuple

import numpy as np
import torch
from torch.utils.data import DataLoader, Dataset

from ..config import TrainConfig, from_deepspeed, parse_duration, to_dict
from ..models import build_model
from ..parallel import dist as ddist
from ..parallel.sampler import ShardSampler
from ..utils import checkpoint as ckpt
from ..utils import fault
from ..utils import mlflow_compat as mlflow
from .schedule import from_config as sched_from_config


@dataclass
class TrainResult:
    model: Any
    history: List[Dict[str, float]] = field(default_factory=list)
    run_id: Optional[str] = None
    best_val_accuracy: float = 0.0
    steps: int = 0
    images_per_sec: float = 0.0
    engine: str = ""
    resumed_epoch: int = 0   # > 0: this run resumed from the checkpoint of that epoch


def _log(msg: str):
    if ddist.get_rank() == 0:
        print(msg, flush=True)


def _uint8_source(ds) -> bool:
    """Can the native loader consume this dataset (fixed-size uint8 HWC + int label, or MDS)?"""
    if hasattr(ds, "native_reader") or hasattr(ds, "shards"):
        return True
    try:
        x, _ = ds[0]
    except Exception:
        return False
    return isinstance(x, np.ndarray) and x.dtype == np.uint8 and x.ndim == 3


def _sample_hw(ds) -> Tuple[int, int, int]:
    if hasattr(ds, "get_item"):
        it = ds.get_item(0)
        img = it["image"]
        a = np.asarray(img)
    else:
        a = np.asarray(ds[0][0])
    if a.ndim == 2:
        a = a[:, :, None]
    return a.shape[0], a.shape[1], a.shape[2]


def _collate_images(batch):
    xs, ys = zip(*batch)
    if isinstance(xs[0], torch.Tensor):
        x = torch.stack(xs)
    else:
        a = np.stack([np.asarray(v) for v in xs])
        if a.dtype == np.uint8:  # uint8 HWC -> float CHW in [0,1] (no Normalize given)
            a = a.transpose(0, 3, 1, 2).astype(np.float32) / 255.0
        x = torch.from_numpy(a)
    return x, torch.tensor(ys, dtype=torch.int64)


def _dict_collate(batch):
    xs = [b["image"] if isinstance(b, dict) else b[0] for b in batch]
    ys = [b["label"] if isinstance(b, dict) else b[1] for b in batch]
    return _collate_images(list(zip(xs, ys)))


def make_loader(ds: Dataset, batch_size: int, shuffle: bool, seed: int, num_workers: int = 0,
                drop_last: bool = False, pin: bool = False):
    if hasattr(ds, "epoch_indices"):  # streaming dataset partitions itself
        return DataLoader(ds, batch_size=batch_size, num_workers=num_workers, collate_fn=_dict_collate,
                          drop_last=drop_last, pin_memory=pin), None
    sampler = ShardSampler(ds, shuffle=shuffle, seed=seed, drop_last=drop_last)
    return DataLoader(ds, batch_size=batch_size, sampler=sampler, num_workers=num_workers,
                      collate_fn=_collate_images, drop_last=drop_last, pin_memory=pin), sampler


class _Native:
    """Adapter: native trainer + loader behind a small common interface."""

    def __init__(self, cfg: TrainConfig, model, ds, dev, steps_per_epoch_hint: int, eval_ds=None):
        from ..data.loader import AugmentSpec, NativeImageLoader
        from ..engine.native_trainer import NativeTrainer, OptimConfig
        h, w, c = _sample_hw(ds)
        s = cfg.data.image_size
        o = cfg.optim
        mean = std = None
        if cfg.data.dataset in ("cifar10", "cifar"):
            from ..data.transforms import CIFAR_MEAN, CIFAR_STD
            mean, std = CIFAR_MEAN, CIFAR_STD
        from ..models.wrappers import FrozenBackboneClassifier
        ar = torch.bfloat16 if cfg.allreduce_dtype == "bf16" else torch.float32
        if isinstance(model, FrozenBackboneClassifier):
            from ..engine.frozen_trainer import FrozenFeatureTrainer
            self.tr = FrozenFeatureTrainer(model, cfg.batch_size, (s, s), dev, o,
                                           label_smoothing=cfg.data.label_smoothing, src_hw=(h, w), mean=mean,
                                           std=std, bucket_cap_mb=cfg.bucket_cap_mb, allreduce_dtype=ar)
        else:
            self.tr = NativeTrainer(model, cfg.batch_size, (s, s), dev,
                                    optim=OptimConfig(o.name, o.lr, o.momentum, 0.0, o.nesterov, o.weight_decay,
                                                      tuple(o.betas), o.eps, o.grad_clip,
                                                      trust_coefficient=o.trust_coefficient),
                                    label_smoothing=cfg.data.label_smoothing, use_graphs=cfg.graphs,
                                    bucket_cap_mb=cfg.bucket_cap_mb, allreduce_dtype=ar,
                                    src_hw=(h, w), mean=mean, std=std, zero_stage=cfg.zero.stage,
                                    cutmix_alpha=cfg.data.cutmix_alpha, seed=cfg.seed)
        if not cfg.data.augment:
            aug = AugmentSpec()
        elif (h, w) == (s, s) and s <= 64:
            aug = AugmentSpec(mode="random_crop", pad=4 if s == 32 else 0, hflip=True)
        elif (h, w) == (s, s):
            aug = AugmentSpec(hflip=True)
        else:
            aug = AugmentSpec(mode="random_resized_crop", hflip=True)
        sampler = None if hasattr(ds, "epoch_indices") else ShardSampler(ds, shuffle=cfg.data.shuffle, seed=cfg.seed,
                                                                          drop_last=True)
        self.sampler = sampler
        self.loader = NativeImageLoader(ds, cfg.batch_size, (h, w), dev, channels=c, augment=aug, out_hw=(s, s),
                                        indices_fn=(lambda e: (sampler.set_epoch(e), sampler.indices().numpy())[1])
                                        if sampler else None, seed=cfg.seed + ddist.get_rank(),
                                        nthreads=max(1, cfg.data.num_workers))
        self.eval_spec = AugmentSpec(mode="center_crop" if (h, w) != (s, s) else "none")
        self.in_hw = (h, w)
        self.batch = cfg.batch_size

    def epoch_batches(self, epoch: int):
        self.loader.set_epoch(epoch)
        return iter(self.loader)

    def steps_per_epoch(self) -> int:
        return len(self.loader)

    def step(self, batch):
        img, lab, boxes, flips = batch
        self.tr.step(img, lab, boxes, flips)

    @staticmethod
    def batch_samples(batch) -> int:
        return int(batch[1].shape[0])

    def set_lr(self, lr):
        self.tr.set_lr(lr)

    def read_metrics(self):
        return self.tr.read_metrics()

    @torch.no_grad()
    def eval_dataset(self, ds) -> Tuple[float, float, int]:
        import torch.nn.functional as F
        from ..data.loader import NativeImageLoader, sample_boxes
        sampler = ShardSampler(ds, shuffle=False, drop_last=False) if not hasattr(ds, "epoch_indices") else None
        h, w, c = _sample_hw(ds)
        ld = NativeImageLoader(ds, self.batch, (h, w), self.tr.dev, channels=c, augment=self.eval_spec,
                               out_hw=(self.tr.prog.H, self.tr.prog.W), drop_last=False,
                               indices_fn=(lambda e: sampler.indices().numpy()) if sampler else None, prefetch=1)
        loss, corr, n = 0.0, 0.0, 0
        seen = set()
        for img, lab, boxes, _ in ld:
            logits = self.tr.evaluate_batch(img, lab, boxes).float()
            loss += F.cross_entropy(logits, lab, reduction="sum").item()
            corr += (logits.argmax(1) == lab).sum().item()
            n += lab.shape[0]
        return loss, corr, n

    @property
    def model(self):
        return getattr(self.tr, "full_model", None) or self.tr.prog.model


class _Autograd:
    def __init__(self, cfg: TrainConfig, model, ds, dev):
        from ..engine.autograd_trainer import AutogradTrainer
        self.tr = AutogradTrainer(model, dev, cfg.optim, label_smoothing=cfg.data.label_smoothing,
                                  bucket_cap_mb=cfg.bucket_cap_mb, zero_stage=cfg.zero.stage,
                                  cutmix_alpha=cfg.data.cutmix_alpha, grad_accum=cfg.grad_accum,
                                  offload_optimizer=cfg.zero.offload_optimizer, offload_param=cfg.zero.offload_param,
                                  bf16=cfg.precision == "bf16", stage3=_stage3_kw(cfg.zero),
                                  allreduce_dtype=torch.bfloat16 if cfg.allreduce_dtype == "bf16" else torch.float32)
        self.loader, self.sampler = make_loader(ds, cfg.batch_size, cfg.data.shuffle, cfg.seed,
                                                num_workers=cfg.data.num_workers if dev.type == "cuda" else 0,
                                                pin=dev.type == "cuda")
        self.batch = cfg.batch_size

    def epoch_batches(self, epoch):
        if self.sampler is not None:
            self.sampler.set_epoch(epoch)
        elif hasattr(self.loader.dataset, "set_epoch"):
            self.loader.dataset.set_epoch(epoch)
        return iter(self.loader)

    def steps_per_epoch(self):
        return len(self.loader)

    def step(self, batch):
        self.tr.step(*batch)

    @staticmethod
    def batch_samples(batch) -> int:
        return int(batch[1].shape[0])

    def set_lr(self, lr):
        self.tr.set_lr(lr)

    def read_metrics(self):
        return self.tr.read_metrics()

    def eval_dataset(self, ds):
        loader, _ = make_loader(ds, self.batch, False, 0)
        loss, corr, n = 0.0, 0, 0
        for x, y in loader:
            l, c = self.tr.eval_batch(x, y)
            loss += l
            corr += c
            n += y.shape[0]
        return loss, float(corr), n

    @property
    def model(self):
        return self.tr.model


def _stage3_kw(z) -> Dict[str, Any]:
    """The ZeRO-3 knobs parallel/fsdp.py honours (DeepSpeed ``stage3_*`` keys)."""
    return {"persistence_threshold": z.stage3_param_persistence_threshold,
            "prefetch_elems": z.stage3_prefetch_bucket_size}


def _pick_engine(cfg: TrainConfig, model, ds, dev) -> str:
    from ..engine.program import supports
    from ..models.wrappers import FrozenBackboneClassifier
    if cfg.engine in ("native", "autograd"):
        return cfg.engine
    if cfg.zero.stage == 3 or cfg.zero.offload_optimizer or cfg.zero.offload_param:
        return "autograd"  # parameter sharding / offload: parallel/fsdp.py on the autograd engine
    if cfg.precision != "bf16":
        return "autograd"  # the native kernels compute in bf16 (fp32 master weights)
    frozen = isinstance(model, FrozenBackboneClassifier) and supports(model.resnet) and \
        not any(p.requires_grad for p in model.resnet.parameters() if p is not None and
                not any(p is q for q in model.resnet.fc.parameters()))
    if dev.type == "cuda" and (supports(model) or frozen) and _uint8_source(ds) and cfg.grad_accum == 1 \
            and (cfg.data.cutmix_alpha == 0 or not frozen):  # CutMix: native box paste + soft-target CE
        return "native"
    return "autograd"


def _apply_env_overrides(cfg: TrainConfig) -> TrainConfig:
    ds_json = os.environ.get("DBX_DEEPSPEED_CONFIG")
    if ds_json and not getattr(cfg, "deepspeed_applied", False):
        cfg = from_deepspeed(json.loads(ds_json), cfg)
    return cfg


def evaluate(runner, dataset) -> Dict[str, float]:
    loss, corr, n = runner.eval_dataset(dataset)
    loss, corr, n = ddist.all_reduce_sum([loss, corr, float(n)])
    return {"val_loss": loss / max(1.0, n), "val_accuracy": corr / max(1.0, n), "val_samples": n}


def train(cfg: Optional[TrainConfig] = None, model: Optional[torch.nn.Module] = None,
          train_dataset: Optional[Dataset] = None, eval_dataset: Optional[Dataset] = None,
          log_mlflow: bool = True, callbacks: Optional[List[Callable]] = None, **overrides) -> TrainResult:
    """Train ``model`` (default: ``build_model(cfg.model)``) on ``train_dataset`` (default: from cfg.data)."""
    cfg = cfg or TrainConfig()
    if overrides:
        from ..config import update_dataclass
        update_dataclass(cfg, overrides)
    cfg = _apply_env_overrides(cfg)
    force_cpu = os.environ.get("DBX_FORCE_CPU") == "1"
    info = ddist.init_distributed(device="cpu" if force_cpu else None)
    dev = info.device
    torch.manual_seed(cfg.seed)
    np.random.seed(cfg.seed)
    if model is None:
        model = build_model(cfg.model, num_classes=cfg.num_classes)
    if train_dataset is None:
        from ..data.datasets import build_dataset
        d = cfg.data
        if d.dataset == "mds":
            from ..data.mds import StreamingDataset
            train_dataset = StreamingDataset(remote=d.mds_remote or None, local=d.mds_local or d.root, shuffle=d.shuffle)
        else:
            train_dataset = build_dataset(d.dataset, d.root, True, None, d.image_size, cfg.num_classes,
                                          d.train_samples or 50 * cfg.batch_size * info.world_size, cfg.seed)
    engine = _pick_engine(cfg, model, train_dataset, dev)
    runner = _Native(cfg, model, train_dataset, dev, 0) if engine == "native" else _Autograd(cfg, model, train_dataset, dev)
    spe = runner.steps_per_epoch()
    total = cfg.max_steps or (parse_duration(cfg.duration, spe, cfg.batch_size) if cfg.duration else spe * cfg.epochs)
    epochs = math.ceil(total / max(1, spe))
    sched = sched_from_config(cfg.sched, cfg.optim.lr, total, spe)
    res = TrainResult(model=model, engine=engine)
    from ..parallel import comm_guard
    watchdog = comm_guard.for_runner(runner, dev)  # a hung / failed peer ends this rank (launcher restarts)
    try:
        # --- resume ----------------------------------------------------------------------------
        start_epoch, step = 0, 0
        if cfg.checkpoint_dir and (cfg.resume == "latest" or int(os.environ.get("DBX_RESTART_COUNT", "0")) > 0):
            path = ckpt.latest_checkpoint(cfg.checkpoint_dir)
            if path:
                st = torch.load(path, map_location="cpu", weights_only=True)
                model.load_state_dict(st["model"])
                _params_changed(runner)
                _restore_trainer_state(runner, st.get("trainer"))
                start_epoch, step = int(st.get("epoch", 0)), int(st.get("step", 0))
                _restore_shard_state(runner, cfg.checkpoint_dir, start_epoch)
                res.history = list(st.get("history", []))
                res.resumed_epoch = start_epoch
                _log(f"[train] resumed from {path} (epoch {start_epoch}, step {step})")
        elif cfg.resume and cfg.resume != "latest":
            st = torch.load(cfg.resume, map_location="cpu", weights_only=True)
            model.load_state_dict(st["model"])
            _params_changed(runner)
        # --- mlflow ------------------------------------------------------------------------------
        is_main = ddist.get_rank() == 0
        if is_main and log_mlflow:
            mlflow.set_experiment(cfg.experiment)
            run = mlflow.start_run(run_name=cfg.run_name or None, nested=mlflow.active_run() is not None)
            res.run_id = run.info.run_id
            mlflow.log_params({"batch_size": cfg.batch_size, "epochs": epochs, "learning_rate": cfg.optim.lr,
                               "model_type": cfg.model, "optimizer": cfg.optim.name, "weight_decay": cfg.optim.weight_decay,
                               "scheduler": cfg.sched.name, "num_gpus": ddist.get_world_size(), "engine": engine,
                               "zero_stage": cfg.zero.stage, "trainer": "dbx_amd"})
        _log(f"[train] engine={engine} world={ddist.get_world_size()} steps/epoch={spe} total_steps={total}")
        best_val, bad_epochs = -1.0, 0
        t_start = time.perf_counter()
        imgs = 0
        stop = False
        for epoch in range(start_epoch, epochs):
            t0 = time.perf_counter()
            n_local = 0  # samples actually stepped this epoch (early stop / short final batch)
            t_wait = t_wall = 0.0  # wall_clock_breakdown: host time waiting for batches / per logging window
            t_mark = time.perf_counter()
            n_win = 0
            it = iter(runner.epoch_batches(epoch))
            while step < total:
                t_b = time.perf_counter()
                batch = next(it, None)
                if batch is None:
                    break
                t_wait += time.perf_counter() - t_b
                runner.set_lr(sched(step))
                fault.heartbeat(step)
                if fault.maybe_inject(step):
                    raise FloatingPointError(f"injected NaN loss at step {step}")
                if watchdog is not None:
                    watchdog.step_begin(step)
                runner.step(batch)
                if watchdog is not None:
                    watchdog.step_end()
                step += 1
                n_win += 1
                n_local += runner.batch_samples(batch)
                imgs += cfg.batch_size * ddist.get_world_size()
                if cfg.log_every and step % cfg.log_every == 0:
                    if cfg.wall_clock_breakdown:  # DeepSpeed's per-window timing (synchronised at the window end)
                        if dev.type == "cuda":
                            torch.cuda.synchronize()
                        t_wall = time.perf_counter() - t_mark
                        if is_main:
                            print(f"[wall_clock_breakdown] steps {step - n_win + 1}-{step}: "
                                  f"{1e3 * t_wall / n_win:.2f} ms/step, data wait {1e3 * t_wait / n_win:.2f} ms/step, "
                                  f"compute+sync {1e3 * (t_wall - t_wait) / n_win:.2f} ms/step", flush=True)
                        t_wait, n_win, t_mark = 0.0, 0, time.perf_counter()
                    if is_main:
                        print(f"[TRAINING] [RANK {ddist.get_rank()}] step {step}/{total} (epoch {epoch + 1})", flush=True)
            if watchdog is not None:
                watchdog.step_begin(step)  # the epoch-end collectives are bounded too
            loss_sum, correct = runner.read_metrics()
            loss_sum, correct, n = ddist.all_reduce_sum([loss_sum, correct, float(n_local)])
            if watchdog is not None:
                watchdog.step_end()
            if not fault.check_finite(loss_sum):
                raise FloatingPointError(f"non-finite training loss in epoch {epoch + 1}")
            rec = {"epoch": epoch + 1, "train_loss": loss_sum / max(1.0, n), "train_accuracy": correct / max(1.0, n),
                   "learning_rate": sched(max(0, step - 1)), "epoch_time_s": time.perf_counter() - t0}
            if eval_dataset is not None and cfg.eval_every and (epoch + 1) % cfg.eval_every == 0:
                rec.update(evaluate(runner, eval_dataset))
            res.history.append(rec)
            if is_main:
                _log(f"Epoch [{epoch + 1}/{epochs}], Loss: {rec['train_loss']:.4f}, Accuracy: {rec['train_accuracy']:.4f}"
                     + (f", Val Loss: {rec['val_loss']:.4f}, Val Accuracy: {rec['val_accuracy']:.4f}" if "val_loss" in rec else ""))
                if log_mlflow:
                    mlflow.log_metrics({k: v for k, v in rec.items() if k != "epoch"}, step=epoch + 1)
            for cb in callbacks or []:
                cb(epoch + 1, rec, runner)
            if cfg.checkpoint_dir and cfg.checkpoint_every and (epoch + 1) % cfg.checkpoint_every == 0:
                _sync_master(runner)  # every rank (collective): ZeRO shards -> full fp32 parameters
                _save_shard_state(runner, cfg.checkpoint_dir, epoch + 1)  # every rank: its ZeRO shard
            if cfg.checkpoint_dir and is_main and cfg.checkpoint_every and (epoch + 1) % cfg.checkpoint_every == 0:
                ckpt.save_checkpoint(cfg.checkpoint_dir, runner.model, None, epoch + 1, step=step,
                                     trainer=_trainer_state(runner), history=res.history, config=json.dumps(to_dict(cfg)))
            ddist.barrier()
            if "val_accuracy" in rec:
                res.best_val_accuracy = max(res.best_val_accuracy, rec["val_accuracy"])
                if cfg.patience:
                    if rec["val_accuracy"] > best_val:
                        best_val, bad_epochs = rec["val_accuracy"], 0
                    else:
                        bad_epochs += 1
                    stop = bool(ddist.broadcast_object(bad_epochs >= cfg.patience))
            if stop:
                _log(f"[train] early stopping after epoch {epoch + 1} (patience {cfg.patience})")
                break
            if step >= total:
                break
        if torch.cuda.is_available() and dev.type == "cuda":
            torch.cuda.synchronize()
    finally:
        # every exit (an exception out of a step included): a live watchdog would otherwise end the
        # process DBX_COMM_TIMEOUT seconds later, under a caller that caught the exception
        if watchdog is not None:
            watchdog.close()
    el = time.perf_counter() - t_start
    _sync_master(runner)  # the returned / logged model holds the full parameters on every rank
    res.steps = step
    res.images_per_sec = imgs / el if el > 0 else 0.0
    res.model = runner.model
    if is_main and log_mlflow:
        mlflow.log_metric("images_per_sec", res.images_per_sec)
        mlflow.pytorch.log_model(res.model, cfg.model_name or "model")
        mlflow.log_dict({"history": res.history}, "training_history.json")
        mlflow.end_run()
    return res


def _sync_master(runner) -> None:
    f = getattr(runner.tr, "sync_master", None)
    if f is not None:
        f()


def _params_changed(runner) -> None:
    f = getattr(runner.tr, "params_changed", None)
    if f is not None:
        f()


def _trainer_state(runner) -> Dict[str, Any]:
    tr = runner.tr
    if hasattr(tr, "prog") and hasattr(tr, "mom"):  # native: flat optimizer state
        st = {"kind": "native", "mom": tr.mom.detach().cpu(), "step_count": tr.step_count}
        if tr.mom2 is not None:
            st["mom2"] = tr.mom2.detach().cpu()
        return st
    if getattr(tr, "opt", None) is not None:
        return {"kind": "torch", "optimizer": ckpt.clean_state_dict(tr.opt.state_dict())}
    return {}


def _shard_path(d: str, epoch: int) -> str:
    return os.path.join(d, f"zero_shard-{epoch}-rank{ddist.get_rank()}-of{ddist.get_world_size()}.pt")


def _sharded(runner):
    """(save, load) of this rank's sharded optimizer state (ZeRO-1/2 or ZeRO-3), if any."""
    tr = runner.tr
    if getattr(tr, "sharded", False):
        return tr.ddp.optim_state_dict, tr.ddp.load_optim_state_dict
    z = getattr(tr, "zero", None)
    if z is not None:
        return z.state_dict, z.load_state_dict
    return None


def _save_shard_state(runner, d: str, epoch: int) -> None:
    sh = _sharded(runner)
    if sh is None:
        return
    os.makedirs(d, exist_ok=True)
    torch.save(sh[0](), _shard_path(d, epoch))


def _restore_shard_state(runner, d: str, epoch: int) -> None:
    """Each rank reloads its own optimizer shard (the rank-0 checkpoint holds only rank 0's)."""
    sh = _sharded(runner)
    if sh is None:
        return
    p = _shard_path(d, epoch)
    if not os.path.exists(p):
        _log(f"[train] warning: no optimizer shard {p}; sharded optimizer state starts fresh")
        return
    sh[1](torch.load(p, map_location="cpu", weights_only=True))


def _restore_trainer_state(runner, st):
    if not st:
        return
    tr = runner.tr
    if st.get("kind") == "native" and hasattr(tr, "mom"):
        tr.mom.copy_(st["mom"])
        if "mom2" in st and tr.mom2 is not None:
            tr.mom2.copy_(st["mom2"])
        tr.step_count = int(st.get("step_count", 0))
    elif st.get("kind") == "torch" and getattr(tr, "opt", None) is not None:
        tr.opt.load_state_dict(st["optimizer"])
