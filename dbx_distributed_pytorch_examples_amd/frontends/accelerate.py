"""HF-Accelerate-style API (`04_accelerate/01_cifar_accelerate.ipynb`) over our process group / DDP.

``Accelerator().prepare(model, optimizer, train_loader, eval_loader, scheduler)`` moves the model to
this rank's GPU (channels_last), wraps it in the flat-bucket DDP, re-shards the loaders with
``ShardSampler`` (their batches then arrive on the device) and returns them; ``backward(loss)`` runs autograd and finishes the bucket
all-reduces; ``gather`` / ``reduce`` are packed collectives; ``log`` forwards to the MLflow-compat
tracker (``log_with="mlflow"``). bf16 autocast is enabled by ``mixed_precision="bf16"``.

On a GPU, ``prepare`` puts a supported ResNet (the notebook's ``resnet50`` with a new ``fc``,
`04_accelerate/01_cifar_accelerate.ipynb:475-503`) on the native HIP kernels by default:
:func:`~dbx_distributed_pytorch_examples_amd.engine.native_module.native_module` compiles it for
the first training batch's shape (engine field ``native_frontends=0`` or ``mixed_precision="no"`` keep the
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
from ..engine_config import EngineConfig


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
    """The subset of ``accelerate.Accelerator`` (HF Accelerate 1.x) the reference notebook and
    typical single-node loops use, with the same method and argument names
    (``tests/test_accelerate_api.py`` checks them against the installed package). Differences:
    ``mixed_precision`` defaults to ``"bf16"`` (the MI355X compute dtype), and a supported ResNet
    is put on the native HIP kernels by ``prepare`` (module docstring)."""

    def __init__(self, device_placement: bool = True, split_batches: bool = False,
                 mixed_precision: Optional[str] = "bf16", gradient_accumulation_steps: int = 1, cpu: bool = False,
                 log_with: Optional[str] = None, **_):
        self.info = ddist.init_distributed(device="cpu" if cpu else None)
        self._device = self.info.device
        self._mixed_precision = mixed_precision or "no"
        self.log_with = log_with
        self.device_placement = device_placement
        self.split_batches = split_batches
        self.gradient_accumulation_steps = max(1, int(gradient_accumulation_steps))
        self._models: List[DistributedDataParallel] = []
        self._trackers = False
        self._step = 0
        self._trigger = False

    @property
    def device(self) -> torch.device:
        return self._device

    @property
    def mixed_precision(self) -> str:
        return self._mixed_precision

    @property
    def distributed_type(self) -> str:
        return "MULTI_GPU" if self.num_processes > 1 and self.device.type == "cuda" else (
            "MULTI_CPU" if self.num_processes > 1 else "NO")

    @property
    def use_distributed(self) -> bool:
        return self.num_processes > 1

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

    @property
    def is_last_process(self) -> bool:
        return ddist.get_rank() == self.num_processes - 1

    @property
    def sync_gradients(self) -> bool:
        """True on the micro-step that completes a gradient-accumulation window."""
        return self._step % self.gradient_accumulation_steps == 0

    def print(self, *args, **kwargs):
        if self.is_main_process:
            print(*args, **kwargs)

    def _prep_one(self, obj):
        if isinstance(obj, torch.nn.Module):
            import os
            from ..engine.native_module import NativeResNet, native_module
            from ..engine.program import supports
            if isinstance(obj, NativeResNet):
                return obj  # on the device already; gradients all-reduced by its own backward
            if (self.device.type == "cuda" and self.mixed_precision == "bf16" and supports(obj)
                    and EngineConfig.current().native_frontends):
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
            return _DeviceLoader(dl, self.device) if (self.device.type != "cpu" and self.device_placement) else dl
        return obj  # schedulers etc.

    def prepare(self, *args, device_placement=None):
        out = tuple(self._prep_one(o) for o in args)
        return out[0] if len(out) == 1 else out

    def autocast(self, autocast_handler=None):
        enabled = self.device.type == "cuda" and self.mixed_precision == "bf16"
        return torch.autocast(self.device.type, dtype=torch.bfloat16, enabled=enabled)

    def backward(self, loss: torch.Tensor, **kwargs) -> None:
        if self.gradient_accumulation_steps > 1:
            loss = loss / self.gradient_accumulation_steps
        loss.backward(**kwargs)
        for m in self._models:
            m.finish_gradient_sync()

    @contextlib.contextmanager
    def accumulate(self, *models):
        """Gradient accumulation window: gradients are synchronised on the window's last micro-step."""
        self._step += 1
        if self.sync_gradients:
            yield
        else:
            with contextlib.ExitStack() as st:
                for m in models:
                    if hasattr(m, "no_sync"):
                        st.enter_context(m.no_sync())
                yield

    def clip_grad_norm_(self, parameters, max_norm, norm_type=2):
        for m in self._models:
            m.finish_gradient_sync()
        return torch.nn.utils.clip_grad_norm_(parameters, max_norm, norm_type=norm_type)

    def gather(self, tensor: torch.Tensor) -> torch.Tensor:
        t = torch.as_tensor(tensor, device=self.device)
        if ddist.get_world_size() == 1:
            return t.reshape(1, *t.shape) if t.dim() == 0 else t
        import torch.distributed as dist
        parts = [torch.empty_like(t.reshape(-1) if t.dim() == 0 else t) for _ in range(ddist.get_world_size())]
        dist.all_gather(parts, t.reshape(-1) if t.dim() == 0 else t)
        return torch.cat(parts)

    def gather_for_metrics(self, input_data, use_gather_object: bool = False):
        if use_gather_object or not isinstance(input_data, torch.Tensor):
            if ddist.get_world_size() == 1:
                return input_data if isinstance(input_data, list) else [input_data]
            import torch.distributed as dist
            out = [None] * ddist.get_world_size()
            dist.all_gather_object(out, input_data)
            return [v for part in out for v in (part if isinstance(part, list) else [part])]
        return self.gather(input_data)

    def pad_across_processes(self, tensor, dim=0, pad_index=0, pad_first=False):
        t = torch.as_tensor(tensor, device=self.device)
        if ddist.get_world_size() == 1:
            return t
        n = int(max(self.gather(torch.tensor([t.shape[dim]], device=self.device)).tolist()))
        if t.shape[dim] == n:
            return t
        shape = list(t.shape)
        shape[dim] = n - t.shape[dim]
        pad = torch.full(shape, pad_index, dtype=t.dtype, device=t.device)
        return torch.cat([pad, t] if pad_first else [t, pad], dim=dim)

    def reduce(self, tensor: torch.Tensor, reduction: str = "sum", scale: float = 1.0) -> torch.Tensor:
        t = torch.as_tensor(tensor, device=self.device).clone()
        ddist.all_reduce_tensor_(t)
        if reduction == "mean":
            t /= ddist.get_world_size()
        return t * scale if scale != 1.0 else t

    def wait_for_everyone(self) -> None:
        ddist.barrier()

    @contextlib.contextmanager
    def main_process_first(self):
        if not self.is_main_process:
            self.wait_for_everyone()
        yield
        if self.is_main_process:
            self.wait_for_everyone()

    @contextlib.contextmanager
    def local_main_process_first(self):
        with self.main_process_first():
            yield

    def split_between_processes(self, inputs, apply_padding: bool = False):
        """Context manager (as in Accelerate) yielding this rank's contiguous slice of ``inputs``."""
        n, r = self.num_processes, self.process_index

        @contextlib.contextmanager
        def _cm():
            k = len(inputs)
            per, extra = divmod(k, n)
            lo = r * per + min(r, extra)
            hi = lo + per + (1 if r < extra else 0)
            part = inputs[lo:hi]
            if apply_padding and extra and r >= extra and k:
                part = part + inputs[-1:] if isinstance(part, list) else torch.cat([part, inputs[-1:]])
            yield part
        return _cm()

    def unwrap_model(self, model, keep_fp32_wrapper: bool = True, keep_torch_compile: bool = True):
        return unwrap(model)

    def get_state_dict(self, model, unwrap: bool = True):
        m = self.unwrap_model(model) if unwrap else model
        return {k: v.detach().cpu() for k, v in m.state_dict().items()}

    def init_trackers(self, project_name: str, config: Optional[dict] = None, init_kwargs: Optional[dict] = None):
        if self.log_with == "mlflow" and self.is_main_process:
            mlflow.set_experiment(project_name)
            if mlflow.active_run() is None:
                mlflow.start_run()
            if config:
                mlflow.log_params(config)
            self._trackers = True

    def log(self, values: dict, step: Optional[int] = None, log_kwargs: Optional[dict] = None) -> None:
        if self._trackers and self.is_main_process:
            mlflow.log_metrics({k: float(v) for k, v in values.items()}, step=step)

    def end_training(self) -> None:
        if self._trackers and self.is_main_process and mlflow.active_run() is not None:
            mlflow.end_run()
        self._trackers = False

    def save(self, obj, f, safe_serialization: bool = False) -> None:
        if self.is_main_process:
            if safe_serialization:
                from safetensors.torch import save_file
                save_file({k: v.contiguous() for k, v in obj.items()}, f)
            else:
                torch.save(obj, f)

    def save_state(self, output_dir: Optional[str] = None, safe_serialization: bool = True, **_):
        """Every prepared model's state dict and the RNG state under ``output_dir`` (rank 0 writes)."""
        import os
        output_dir = output_dir or "accelerate_state"
        if self.is_main_process:
            os.makedirs(output_dir, exist_ok=True)
            for i, m in enumerate(self._models):
                torch.save(self.get_state_dict(m), os.path.join(output_dir, f"model_{i}.bin"))
            torch.save({"torch": torch.get_rng_state(), "step": self._step}, os.path.join(output_dir, "random_states.pkl"))
        self.wait_for_everyone()
        return output_dir

    def load_state(self, input_dir: Optional[str] = None, load_kwargs: Optional[dict] = None, **_):
        import os
        input_dir = input_dir or "accelerate_state"
        for i, m in enumerate(self._models):
            sd = torch.load(os.path.join(input_dir, f"model_{i}.bin"), map_location="cpu", weights_only=True)
            self.unwrap_model(m).load_state_dict(sd)
        st = torch.load(os.path.join(input_dir, "random_states.pkl"), map_location="cpu", weights_only=True)
        torch.set_rng_state(st["torch"])
        self._step = int(st["step"])

    def free_memory(self, *objects):
        import gc
        self._models.clear()
        gc.collect()
        if torch.cuda.is_available():
            torch.cuda.empty_cache()
        return [None for _ in objects]

    def set_trigger(self):
        self._trigger = True

    def check_trigger(self) -> bool:
        flag = self.reduce(torch.tensor(float(self._trigger)), reduction="sum")
        if float(flag) > 0:
            self._trigger = False
            return True
        return False

    @contextlib.contextmanager
    def no_sync(self, model):
        with model.no_sync():
            yield


CIFAR10_CLASSES = ("plane", "car", "bird", "cat", "deer", "dog", "frog", "horse", "ship", "truck")


def broadcast_run_id(run_id: Optional[str], accelerator: Accelerator) -> Optional[str]:
    """Rank 0's MLflow run id on every rank (the notebook sends it as a length + code-point tensor
    pair, `04_accelerate/01_cifar_accelerate.ipynb:764-778`; here one object broadcast)."""
    if accelerator.num_processes == 1:
        return run_id
    return ddist.broadcast_object(run_id if accelerator.is_main_process else None)


def train_model(run_id: Optional[str] = None, *, accelerator: Accelerator, model, optimizer, scheduler, criterion,
                train_loader, test_loader, config: dict, classes=CIFAR10_CLASSES):
    """The notebook's ``train_model(run_id=None) -> (history, run_id)``
    (`04_accelerate/01_cifar_accelerate.ipynb:553-790`) over prepared objects: per epoch a training
    pass and an evaluation pass, metrics summed across ranks, ``CosineAnnealingLR``-style
    ``scheduler.step()`` per epoch, then on rank 0:

    * MLflow metrics ``train_loss`` / ``train_accuracy`` / ``test_loss`` / ``test_accuracy`` /
      ``learning_rate`` (step = epoch), also sent through ``accelerator.log``;
    * the checkpoint dict ``{epoch, model_state_dict, optimizer_state_dict, scheduler_state_dict,
      test_accuracy}`` as ``checkpoints/epoch_{k}`` every ``config["save_every"]`` epochs and at the end;
    * the best model as ``best_model`` + ``best_model/metadata.json`` (epoch, accuracy, config, classes);
    * ``training_history.json`` with keys train_loss / train_acc / test_loss / test_acc / lr.

    A new MLflow run is started when ``run_id`` is None (parameters logged), otherwise the active
    run continues. The run id is broadcast from rank 0, so every rank returns the same
    ``(history, run_id)``. Losses are sample-weighted means (the notebook divides a sum of batch
    means by the dataset size); per-batch statistics accumulate on the device (no per-step host sync).
    """
    acc = accelerator
    params = {"model_type": "ResNet50", "batch_size": config["batch_size"], "epochs": config["num_epochs"],
              "learning_rate": config["learning_rate"], "weight_decay": config["weight_decay"], "optimizer": "Adam",
              "scheduler": "CosineAnnealingLR", "num_gpus": acc.num_processes}
    if acc.is_main_process:
        if run_id is None:
            run_id = (mlflow.active_run() or mlflow.start_run()).info.run_id
        elif mlflow.active_run() is None:
            mlflow.start_run(run_id=run_id)  # resume the given run
        mlflow.log_params(params)
    acc.wait_for_everyone()
    history = {"train_loss": [], "train_acc": [], "test_loss": [], "test_acc": [], "lr": []}
    best = 0.0
    save_every = int(config.get("save_every", 1))
    for epoch in range(config["num_epochs"]):
        model.train()
        sums = torch.zeros(3, device=acc.device)
        for inputs, targets in train_loader:
            optimizer.zero_grad()
            with acc.autocast():
                outputs = model(inputs)
                loss = criterion(outputs.float(), targets)
            acc.backward(loss)
            optimizer.step()
            sums += torch.stack([loss.detach().float() * targets.shape[0],
                                 (outputs.detach().argmax(1) == targets).sum().float(),
                                 torch.tensor(float(targets.shape[0]), device=sums.device)])
        tl, tc, tn = acc.reduce(sums).tolist()
        model.eval()
        ev = torch.zeros(3, device=acc.device)
        with torch.no_grad():
            for inputs, targets in test_loader:
                with acc.autocast():
                    outputs = model(inputs)
                ev += torch.stack([criterion(outputs.float(), targets).float() * targets.shape[0],
                                   (outputs.argmax(1) == targets).sum().float(),
                                   torch.tensor(float(targets.shape[0]), device=ev.device)])
        el, ec, en = acc.reduce(ev).tolist()
        train_loss, train_accuracy = tl / max(1.0, tn), 100.0 * tc / max(1.0, tn)
        test_loss, test_accuracy = el / max(1.0, en), 100.0 * ec / max(1.0, en)
        current_lr = scheduler.get_last_lr()[0]
        scheduler.step()
        metrics = {"train_loss": train_loss, "train_accuracy": train_accuracy, "test_loss": test_loss,
                   "test_accuracy": test_accuracy, "learning_rate": current_lr}
        if acc.is_main_process:
            for k, v in (("train_loss", train_loss), ("train_acc", train_accuracy), ("test_loss", test_loss),
                         ("test_acc", test_accuracy), ("lr", current_lr)):
                history[k].append(v)
            mlflow.log_metrics(metrics, step=epoch)
        acc.log(metrics)
        acc.print(f"[Rank {acc.process_index}] Epoch {epoch + 1}/{config['num_epochs']} - Train Loss: {train_loss:.4f}, "
                  f"Train Acc: {train_accuracy:.2f}%, Test Loss: {test_loss:.4f}, Test Acc: {test_accuracy:.2f}%")
        acc.wait_for_everyone()
        if acc.is_main_process:
            unwrapped = acc.unwrap_model(model)
            if (epoch + 1) % save_every == 0 or epoch == config["num_epochs"] - 1:
                ck = {"epoch": epoch + 1, "model_state_dict": unwrapped.state_dict(),
                      "optimizer_state_dict": optimizer.state_dict(), "scheduler_state_dict": scheduler.state_dict(),
                      "test_accuracy": test_accuracy}
                mlflow.pytorch.log_state_dict(ck, f"checkpoints/epoch_{epoch + 1}")
            if test_accuracy > best:
                best = test_accuracy
                mlflow.pytorch.log_model(unwrapped, "best_model")
                mlflow.log_dict({"epoch": epoch + 1, "test_accuracy": test_accuracy, "config": config,
                                 "classes": list(classes)}, "best_model/metadata.json")
    if acc.is_main_process:
        mlflow.log_dict(history, "training_history.json")
    acc.end_training()
    acc.wait_for_everyone()
    run_id = broadcast_run_id(run_id, acc)
    if acc.is_main_process and mlflow.active_run() is not None:
        mlflow.end_run()
    return history, run_id
