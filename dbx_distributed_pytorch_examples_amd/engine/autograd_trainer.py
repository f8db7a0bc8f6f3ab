"""Generic training step for any ``nn.Module`` (models the native ResNet program does not cover:
the MNIST ``Net``, frozen-backbone heads, Composer-style models, user modules) and for CPU hosts.

Stock autograd + our flat-bucket DDP (``parallel.ddp``) + bf16 autocast on the GPU
(channels_last memory format), torch optimizers (or the flat ZeRO optimizer). Loss: the model's
own ``loss(outputs, batch)`` if it has one (Composer convention), NLL for log-probability outputs
(the reference MNIST ``Net`` ends in ``log_softmax``, `01_basic_torch_distributor.py:91,99`), else
cross-entropy with optional label smoothing; optional CutMix on the batch (Composer algorithm).
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..parallel.ddp import DistributedDataParallel, flat_view, unwrap


class LARS(torch.optim.Optimizer):
    """SGD-momentum with layer-wise adaptive rate scaling (You et al., large-batch ImageNet): for every
    tensor with ndim > 1, g <- eta*|w|/(|g| + wd*|w|) * (g + wd*w); 1-d tensors (BN, biases) take the
    plain gradient without decay. Same math as the native ``lars_scale`` + ``sgd_step`` kernels."""

    def __init__(self, params, lr, momentum=0.9, weight_decay=0.0, trust_coefficient=0.001, nesterov=False):
        super().__init__(params, dict(lr=lr, momentum=momentum, weight_decay=weight_decay, eta=trust_coefficient,
                                      nesterov=nesterov))

    @torch.no_grad()
    def step(self, closure=None):
        for grp in self.param_groups:
            for p in grp["params"]:
                if p.grad is None:
                    continue
                d = p.grad
                if p.ndim > 1:
                    wn, gn = p.norm(), d.norm()
                    trust = torch.where((wn > 0) & (gn > 0), grp["eta"] * wn / (gn + grp["weight_decay"] * wn),
                                        torch.ones_like(wn))
                    d = (d + grp["weight_decay"] * p) * trust
                st = self.state[p]
                if grp["momentum"]:
                    buf = st.get("momentum_buffer")
                    if buf is None:
                        buf = st["momentum_buffer"] = d.clone()
                    else:
                        buf.mul_(grp["momentum"]).add_(d)
                    d = d + grp["momentum"] * buf if grp["nesterov"] else buf
                p.add_(d, alpha=-grp["lr"])


def build_torch_optimizer(params, o):
    if o.name == "lars":
        return LARS(params, lr=o.lr, momentum=o.momentum, weight_decay=o.weight_decay,
                    trust_coefficient=getattr(o, "trust_coefficient", 0.001), nesterov=o.nesterov)
    if o.name == "sgd":
        return torch.optim.SGD(params, lr=o.lr, momentum=o.momentum, nesterov=o.nesterov, weight_decay=o.weight_decay)
    if o.name == "adam":
        return torch.optim.Adam(params, lr=o.lr, betas=tuple(o.betas), eps=o.eps, weight_decay=o.weight_decay)
    if o.name == "adamw":
        return torch.optim.AdamW(params, lr=o.lr, betas=tuple(o.betas), eps=o.eps, weight_decay=o.weight_decay)
    raise ValueError(f"unknown optimizer {o.name!r}")


def cutmix(x: torch.Tensor, y: torch.Tensor, num_classes: int, alpha: float, gen: Optional[torch.Generator] = None):
    """CutMix (Composer ``CutMix(alpha)``, `03_composer/01_cifar_composer_resnet.ipynb:430`): paste a
    box from a permuted batch, mix one-hot targets by the pasted area."""
    lam = torch.distributions.Beta(alpha, alpha).sample().item() if alpha > 0 else 1.0
    B, _, H, W = x.shape
    perm = torch.randperm(B, device=x.device)
    rh, rw = int(H * math.sqrt(1 - lam)), int(W * math.sqrt(1 - lam))
    cy, cx = torch.randint(0, H, (1,)).item(), torch.randint(0, W, (1,)).item()
    y0, y1 = max(cy - rh // 2, 0), min(cy + rh // 2, H)
    x0, x1 = max(cx - rw // 2, 0), min(cx + rw // 2, W)
    x = x.clone()
    x[:, :, y0:y1, x0:x1] = x[perm, :, y0:y1, x0:x1]
    lam = 1 - (y1 - y0) * (x1 - x0) / (H * W)
    t = F.one_hot(y, num_classes).float()
    return x, lam * t + (1 - lam) * t[perm]


def soft_cross_entropy(logits: torch.Tensor, target: torch.Tensor, smoothing: float = 0.0) -> torch.Tensor:
    if smoothing:
        target = target * (1 - smoothing) + smoothing / target.shape[1]
    return -(target * F.log_softmax(logits.float(), 1)).sum(1).mean()


class AutogradTrainer:
    def __init__(self, model: nn.Module, device: torch.device, optim, label_smoothing: float = 0.0,
                 bucket_cap_mb: float = 64.0, channels_last: bool = True, zero_stage: int = 0,
                 cutmix_alpha: float = 0.0, grad_accum: int = 1, allreduce_dtype=torch.float32,
                 offload_optimizer: bool = False, offload_param: bool = False, bf16: bool = True,
                 stage3: Optional[dict] = None):
        self.dev = device
        self.bf16 = bool(bf16) and device.type == "cuda"  # autocast bf16 (DeepSpeed bf16.enabled)
        self.model = model.to(device)
        if device.type == "cuda" and channels_last:
            self.model = self.model.to(memory_format=torch.channels_last)
        self.sharded = zero_stage == 3 or offload_optimizer or offload_param
        if self.sharded:  # ZeRO-3: parameters, gradients and optimizer state sharded (parallel/fsdp.py)
            from ..parallel.fsdp import ShardedDataParallel
            self.ddp = ShardedDataParallel(self.model, optim, offload_optimizer=offload_optimizer,
                                           offload_param=offload_param, **(stage3 or {}))
            zero_stage = 0
        else:
            from .native_module import NativeResNet
            # a native_module inside averages its own gradients (overlapped, per backward segment)
            own_sync = any(isinstance(m, NativeResNet) for m in self.model.modules())
            self.ddp = DistributedDataParallel(self.model, bucket_cap_mb=bucket_cap_mb, allreduce_dtype=allreduce_dtype,
                                               gradient_sync=not own_sync)
        self.world = self.ddp.world
        self.o = optim
        self.smoothing = label_smoothing
        self.cutmix_alpha = cutmix_alpha
        self.grad_accum = max(1, grad_accum)
        self.num_classes = getattr(unwrap(model), "num_classes", None)
        self.zero = None
        params = [p for p in self.model.parameters() if p.requires_grad]
        if self.sharded:
            self.opt = None
        elif zero_stage and params:
            from ..parallel.zero import ZeroShardedOptimizer
            # ZeRO over the DDP flat gradient buffer: master = flat copy of params in the same order
            self._zero_master = torch.zeros_like(self.ddp.flat.buffer)
            for p, off in zip(self.ddp._params, self.ddp.flat.offsets):
                flat_view(self._zero_master, off, p).copy_(p.detach())  # the gradients' memory order
            self.zero = ZeroShardedOptimizer(self._zero_master, self.ddp.flat.buffer, optim, stage=zero_stage,
                                             grad_scale=1.0)  # DDP already averaged
            self.opt = None
        else:
            self.opt = build_torch_optimizer(params, optim) if params else None
        self.micro = 0
        self.loss_sum = torch.zeros((), device=device)
        self.correct = torch.zeros((), device=device)
        self.count = 0

    def set_lr(self, lr: float):
        self.o.lr = lr
        if self.opt is not None:
            for g in self.opt.param_groups:
                g["lr"] = lr

    def _loss(self, out, x, y, target=None):
        m = unwrap(self.model)
        if hasattr(m, "loss") and callable(m.loss) and target is None:
            return m.loss(out, (x, y), label_smoothing=self.smoothing) if "label_smoothing" in m.loss.__code__.co_varnames \
                else m.loss(out, (x, y))
        if target is not None:
            return soft_cross_entropy(out, target, self.smoothing)
        if getattr(m, "outputs_log_probs", False) or isinstance(m, _log_prob_types()):
            return F.nll_loss(out.float(), y)
        return F.cross_entropy(out.float(), y, label_smoothing=self.smoothing)

    def step(self, x: torch.Tensor, y: torch.Tensor) -> None:
        self.model.train()
        x = x.to(self.dev, non_blocking=True)
        y = y.to(self.dev, non_blocking=True)
        if self.dev.type == "cuda" and x.dim() == 4:
            x = x.contiguous(memory_format=torch.channels_last)
        target = None
        if self.cutmix_alpha > 0 and self.num_classes:
            x, target = cutmix(x, y, self.num_classes, self.cutmix_alpha)
        last_micro = (self.micro + 1) % self.grad_accum == 0
        ctx = self.ddp.no_sync() if not last_micro else _null()
        with ctx:
            with torch.autocast(self.dev.type, dtype=torch.bfloat16, enabled=self.bf16):
                out = self.ddp(x) if not _is_composer(self.model) else self.ddp((x, y))
            loss = self._loss(out, x, y, target) / self.grad_accum
            loss.backward()
        self.loss_sum += loss.detach().float() * self.grad_accum * y.shape[0]
        self.correct += (out.detach().argmax(1) == y).sum()
        self.count += y.shape[0]
        self.micro += 1
        if not last_micro:
            return
        self.ddp.finish_gradient_sync()
        if self.sharded:
            self.ddp.optimizer_step()
            self.ddp.zero_grad()
            return
        if self.o.grad_clip and self.zero is None:
            torch.nn.utils.clip_grad_norm_([p for p in self.model.parameters() if p.grad is not None], self.o.grad_clip)
        if self.zero is not None:
            self.zero.step(grads_already_reduced=True)
            with torch.no_grad():
                for p, off in zip(self.ddp._params, self.ddp.flat.offsets):
                    p.copy_(flat_view(self._zero_master, off, p))
        elif self.opt is not None:
            self.opt.step()
        self.ddp.zero_grad()

    def read_metrics(self, reset: bool = True) -> Tuple[float, float]:
        if self.sharded:  # epoch end (all ranks): full parameters for evaluation / rank-0 checkpoints
            self.ddp.gather_full_params()
        loss, corr = float(self.loss_sum.item()), float(self.correct.item())
        if reset:
            self.loss_sum.zero_()
            self.correct.zero_()
            self.count = 0
        return loss, corr

    @torch.no_grad()
    def eval_batch(self, x, y) -> Tuple[float, int]:
        self.model.eval()
        x, y = x.to(self.dev), y.to(self.dev)
        if self.dev.type == "cuda" and x.dim() == 4:
            x = x.contiguous(memory_format=torch.channels_last)
        with torch.autocast(self.dev.type, dtype=torch.bfloat16, enabled=self.bf16):
            out = self.model((x, y)) if _is_composer(self.model) else self.model(x)
        out = out.float()
        m = unwrap(self.model)
        if isinstance(m, _log_prob_types()):
            loss = F.nll_loss(out, y, reduction="sum")
        else:
            loss = F.cross_entropy(out, y, reduction="sum")
        return float(loss.item()), int((out.argmax(1) == y).sum().item())


def _log_prob_types():
    from ..models.mnist import Net
    return (Net,)


def _is_composer(model) -> bool:
    from ..models.wrappers import ComposerResNet50
    return isinstance(unwrap(model), ComposerResNet50)


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
