"""Drop-in autograd module over the native ResNet program: HIP kernels inside a user-written loop.

The reference's Accelerate, Ray and Composer examples train with their OWN loop
(``logits = model(x); loss = criterion(logits, y); loss.backward(); optimizer.step()`` —
`04_accelerate/01_cifar_accelerate.ipynb:553-790`, `05_ray/02_cifar_resnet_pytorch_ray.ipynb:276-333`,
`03_composer/01_cifar_composer_resnet.ipynb:332-346`), so they cannot hand the whole step to
:class:`~.native_trainer.NativeTrainer`. :func:`native_module` wraps a supported ResNet so that
``forward`` runs the native NHWC program (BN statistics in the conv epilogues, BN-apply in the
prologues, ...) and ``backward`` — reached through autograd from whatever loss the loop computes,
soft CutMix targets and label smoothing included — runs the native backward, leaving every
parameter's ``.grad`` as a view of the program's flat gradient buffer. The module's parameters
already ARE views of the program's flat fp32 master, so any torch optimizer steps them in place.

* input: a float NCHW batch, already normalised (what torchvision-style transforms produce);
  batches of another size than the compiled one run through the plain torch module on the same
  parameters (correct, not accelerated);
* gradients: a backward sets ``p.grad`` (or adds into a ``p.grad`` the caller owns); there is no
  accumulation across two backwards into the same view (call ``zero_grad`` between steps, the
  usual loop);
* world size > 1: the flat gradient is all-reduced (averaged) in ONE collective at the end of
  the backward; do not wrap the result in DDP as well (``frontends.accelerate`` knows this);
* on the GPU the program's forward (train / eval) and backward are each captured as a HIP graph
  after two eager calls and replayed (the user loop is otherwise launch-bound at CIFAR sizes);
  the input / dlogits copies into the static buffers and the all-reduce stay outside the graphs.
"""
from __future__ import annotations

import os

from typing import Optional, Tuple

import torch
import torch.distributed as dist
import torch.nn as nn

from .program import ResNetProgram, supports


class _NativeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, anchor, mod):
        ctx.mod = mod
        return mod._native_forward(x)

    @staticmethod
    def backward(ctx, dlogits):
        ctx.mod._native_backward(dlogits)
        return None, torch.zeros_like(ctx.mod._anchor), None


class NativeResNet(nn.Module):
    def __init__(self, model: nn.Module, batch: int, image_hw: Tuple[int, int], device: torch.device,
                 process_group=None):
        super().__init__()
        if not supports(model):
            raise TypeError(f"native_module: {type(model).__name__} is not a supported ResNet")
        self.model = model
        self.prog = ResNetProgram(model, batch, image_hw, device)
        self.prog.build_backward()
        self.pg = process_group
        self.use_graphs = device.type == "cuda" and os.environ.get("DBX_NATIVE_MODULE_GRAPHS", "1") != "0"
        self._graphs = {}  # "fwd_train" / "fwd_eval" / "bwd" -> CUDAGraph
        self._calls = {}
        # autograd needs one leaf that requires grad to route the loss back into _NativeFn
        self._anchor = nn.Parameter(torch.zeros((), device=device), requires_grad=True)
        p = self.prog
        self._grad_views = []
        for prm in model.parameters():
            off = (prm.data_ptr() - p.master.data_ptr()) // 4
            n = prm.numel()
            g = p.grad[off:off + n]
            gv = g.view(prm.shape[0], prm.shape[2], prm.shape[3], prm.shape[1]).permute(0, 3, 1, 2) \
                if prm.dim() == 4 else g.view(prm.shape)
            self._grad_views.append((prm, gv))

    @property
    def module(self) -> nn.Module:
        """the wrapped torch module (``unwrap`` / ``accelerator.unwrap_model`` return it: its parameters
        are the live weights, so it can be saved or logged as a plain model)"""
        return self.model

    def parameters(self, recurse: bool = True):  # the anchor is internal: optimizers see the model's
        return self.model.parameters(recurse)

    def named_parameters(self, prefix: str = "", recurse: bool = True, remove_duplicate: bool = True):
        return self.model.named_parameters(prefix, recurse, remove_duplicate)

    def state_dict(self, *a, **kw):
        return self.model.state_dict(*a, **kw)

    def load_state_dict(self, sd, strict: bool = True):
        with torch.no_grad():
            return self.model.load_state_dict(sd, strict)

    def _apply(self, fn, recurse=True):
        # the parameters are views of the program's flat master (and its HIP buffers live on one
        # device): .to(device / dtype / memory_format), .cuda(), .half() ... must not re-create them
        return self

    def train(self, mode: bool = True):
        super().train(mode)
        self.model.train(mode)
        return self

    # ------------------------------------------------------------------------------
    def forward(self, x: torch.Tensor) -> torch.Tensor:
        p = self.prog
        if x.dim() != 4 or x.shape[0] != p.N or tuple(x.shape[2:]) != (p.H, p.W) or x.shape[1] != p.in_ch:
            return self.model(x)  # another batch size / resolution: the torch module on the same parameters
        if not (torch.is_grad_enabled() and self.training):
            with torch.no_grad():
                return self._native_forward(x)
        return _NativeFn.apply(x, self._anchor, self)

    def _run(self, key: str, fn) -> None:
        """fn() eagerly for the first two calls of this kind, then as a captured graph's replay."""
        if not self.use_graphs:
            fn()
            return
        g = self._graphs.get(key)
        if g is None:
            n = self._calls.get(key, 0)
            if n < 2:
                self._calls[key] = n + 1
                fn()
                return
            torch.cuda.synchronize(self.prog.dev)
            g = torch.cuda.CUDAGraph()
            mode = "thread_local" if (dist.is_available() and dist.is_initialized()) else "global"
            with torch.cuda.graph(g, capture_error_mode=mode):
                fn()
            torch.cuda.synchronize(self.prog.dev)
            self._graphs[key] = g
        g.replay()

    def _fwd_body(self):
        p = self.prog
        p.prepare_weights()
        if p.training:
            p.nbt.add_(1)
        p.forward(compute_grad=False, metrics=False)

    def _native_forward(self, x: torch.Tensor) -> torch.Tensor:
        p = self.prog
        p.training = self.training
        p.x4[..., :p.in_ch].copy_(x.detach().permute(0, 2, 3, 1))  # NCHW float -> NHWC4 bf16
        self._run("fwd_train" if self.training else "fwd_eval", self._fwd_body)
        return p.logits.float()

    def _native_backward(self, dlogits: torch.Tensor) -> None:
        p = self.prog
        p.dlogits.copy_(dlogits)
        self._run("bwd", p.backward)
        world = dist.get_world_size(self.pg) if (dist.is_available() and dist.is_initialized()) else 1
        if world > 1:
            from ..parallel.dist import host_sync_for_gloo
            host_sync_for_gloo(p.grad, self.pg)
            dist.all_reduce(p.grad, group=self.pg)
            p.grad.div_(world)
        for prm, gv in self._grad_views:
            if not prm.requires_grad:
                continue
            if prm.grad is None or prm.grad is gv:
                prm.grad = gv
            else:
                prm.grad.add_(gv)


def native_module(model: nn.Module, batch: int, image_hw: Tuple[int, int] = (224, 224),
                  device: Optional[torch.device] = None, process_group=None) -> NativeResNet:
    """Wrap a supported ResNet (torchvision-layout ResNet-18/34/50/..., the CIFAR-stem ResNet-18)
    for a fixed ``batch`` x ``image_hw``; see the module docstring."""
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    return NativeResNet(model, batch, image_hw, device, process_group)
