"""Flat-bucket data parallelism for arbitrary ``nn.Module`` s (the autograd engine path).

Reference behaviour being replaced: ``DDP(model, device_ids=[local_rank])`` in
`/root/reference/01_torch_distributor/01_basic_torch_distributor.py:289-291` (and the implicit
wraps of Accelerate `accelerator.prepare`, `04_accelerate/01_cifar_accelerate.ipynb:503`, and Ray
`prepare_model`, `05_ray/01_fashion_mnist_pytorch_ray.ipynb:174`) — SURVEY.md §2.5 M2/M3.

Design (MI355X-first rather than a copy of torch DDP's reducer):
* every trainable parameter's ``.grad`` is a VIEW into one contiguous fp32 buffer laid out in
  reverse registration order (≈ gradient-ready order), so a bucket is a slice — no copy-in /
  copy-out, and the optimizer can run one fused kernel over the flat buffer;
* buckets are sized for xGMI (default 64 MiB: 7 point-to-point links per GPU; ring all-reduce is
  per-link bound, so fewer larger messages beat the 25 MiB NVSwitch-era default);
* a bucket's all-reduce is launched (async, RCCL on a GPU, gloo on CPU) from a post-accumulate
  hook as soon as its last gradient lands, overlapping the rest of backward;
* ``no_sync()`` for gradient accumulation, rank-0 parameter/buffer broadcast at construction,
  optional per-step buffer broadcast (torch default ``broadcast_buffers=True``);
* optional bf16 compression of the wire format (``allreduce_dtype``).
"""
from __future__ import annotations

import contextlib
from typing import Dict, List, Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from .dist import host_sync_for_gloo


def flat_view(buf: torch.Tensor, off: int, p: torch.Tensor) -> torch.Tensor:
    """``buf[off:off + p.numel()]`` viewed with ``p``'s shape AND strides when ``p`` is densely packed
    in another memory format (channels-last conv weights): the gradient then obeys autograd's layout
    contract (accumulated in place, no per-step re-layout copy)."""
    if p.is_contiguous() or p.dim() != 4 or not p.is_contiguous(memory_format=torch.channels_last):
        return buf[off:off + p.numel()].view_as(p)
    return buf.as_strided(p.shape, p.stride(), buf.storage_offset() + off)


class FlatGradBuffer:
    """Contiguous gradient storage with params' ``.grad`` as views (reverse order)."""

    def __init__(self, params: List[nn.Parameter], dtype=torch.float32, align: int = 16):
        self.params = params
        device = params[0].device if params else torch.device("cpu")
        offs, total = [], 0
        for p in params:
            offs.append(total)
            total += (p.numel() + align - 1) // align * align
        self.buffer = torch.zeros(max(total, 1), dtype=dtype, device=device)
        self.offsets = offs
        self.numel = total
        self.attach()

    def attach(self):
        for p, o in zip(self.params, self.offsets):
            p.grad = flat_view(self.buffer, o, p)

    def zero_(self):
        self.buffer.zero_()


class DistributedDataParallel(nn.Module):
    def __init__(self, module: nn.Module, process_group=None, bucket_cap_mb: float = 64.0,
                 broadcast_buffers: bool = False, allreduce_dtype: torch.dtype = torch.float32,
                 find_unused_parameters: bool = False, gradient_predivide: bool = True,
                 autocast_dtype: Optional[torch.dtype] = None, gradient_sync: bool = True):
        """``autocast_dtype``: run the wrapped forward under ``torch.autocast`` with that dtype and
        return floating outputs as fp32 (HF Accelerate's ``mixed_precision`` + ``convert_to_fp32``);
        ``gradient_sync=False``: a module that averages its own gradients (``engine.native_module``):
        no broadcast, no bucket all-reduce -- only the flat-buffer / no_sync interface."""
        super().__init__()
        self.module = module
        self.pg = process_group
        self.autocast_dtype = autocast_dtype
        self.world = dist.get_world_size(process_group) if dist.is_available() and dist.is_initialized() else 1
        if not gradient_sync:
            self.world = 1
        self.broadcast_buffers = broadcast_buffers
        self.allreduce_dtype = allreduce_dtype
        self.find_unused = find_unused_parameters
        self.predivide = gradient_predivide
        params = [p for p in module.parameters() if p.requires_grad]
        self._params = list(reversed(params))  # gradient-ready order
        self.flat = FlatGradBuffer(self._params) if self._params else None
        cap = int(bucket_cap_mb * (1 << 20) // 4)
        # buckets: contiguous [lo, hi) ranges in the flat buffer + member params
        self.buckets: List[Dict] = []
        cur = {"lo": 0, "hi": 0, "params": []}
        for p, off in zip(self._params, self.flat.offsets if self.flat else []):
            end = off + (p.numel() + 15) // 16 * 16
            if cur["params"] and end - cur["lo"] > cap:
                self.buckets.append(cur)
                cur = {"lo": off, "hi": off, "params": []}
            cur["params"].append(p)
            cur["hi"] = end
        if cur["params"]:
            self.buckets.append(cur)
        self._p2b = {id(p): i for i, b in enumerate(self.buckets) for p in b["params"]}
        self._pending = [0] * len(self.buckets)
        self._handles: List = []
        self._sync = True
        self._hooks = []
        self.bucket_log: List[int] = []  # launch order of the last round (utils.debug.check_bucket_order)
        if self.world > 1:
            self._broadcast_state()
            for p in self._params:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))
        self._reset_round()

    # ------------------------------------------------------------------------------
    def _broadcast_state(self):
        with torch.no_grad():
            for t in list(self.module.parameters()) + list(self.module.buffers()):
                dist.broadcast(t.data if t.is_contiguous() else t.data.contiguous(), 0, group=self.pg)

    def _reset_round(self):
        self._pending = [len(b["params"]) for b in self.buckets]
        self._handles = []
        self._order: List[int] = []

    def _on_grad(self, p: torch.Tensor):
        if not self._sync or self.world == 1:
            return
        # the flat view may have been replaced (e.g. optimizer.zero_grad(set_to_none=True))
        bi = self._p2b[id(p)]
        self._pending[bi] -= 1
        if self._pending[bi] == 0:
            self._launch(bi)

    def _launch(self, bi: int):
        self._order.append(bi)
        b = self.buckets[bi]
        chunk = self.flat.buffer[b["lo"]:b["hi"]]
        host_sync_for_gloo(chunk, self.pg)
        if self.predivide:
            chunk.div_(self.world)
        if self.allreduce_dtype != chunk.dtype:
            wire = chunk.to(self.allreduce_dtype)
            h = dist.all_reduce(wire, group=self.pg, async_op=True)
            self._handles.append((h, chunk, wire))
        else:
            h = dist.all_reduce(chunk, group=self.pg, async_op=True)
            self._handles.append((h, None, None))

    def finish_gradient_sync(self):
        """Wait for all bucket all-reduces (call before optimizer.step(); idempotent)."""
        if self.world == 1 or not self._sync:
            self._reset_round()
            return
        # buckets whose params got no grad this round (unused params): reduce them now
        for bi, n in enumerate(self._pending):
            if n > 0:
                if not self.find_unused and n != len(self.buckets[bi]["params"]):
                    pass
                self._pending[bi] = 0
                self._launch(bi)
        for h, chunk, wire in self._handles:
            h.wait()
            if chunk is not None:
                chunk.copy_(wire)
        self.bucket_log = list(self._order)
        self._reset_round()

    # ------------------------------------------------------------------------------
    def forward(self, *args, **kw):
        if self.world > 1 and self.broadcast_buffers:
            with torch.no_grad():
                for b in self.module.buffers():
                    dist.broadcast(b, 0, group=self.pg)
        if self.flat is not None:
            # optimizer.zero_grad(set_to_none=True) drops the views: re-zero and re-attach
            buf = self.flat.buffer
            if any(p.grad is None or p.grad.data_ptr() != buf.data_ptr() + 4 * o
                   for p, o in zip(self._params, self.flat.offsets)):
                self.flat.zero_()
                self.flat.attach()
        self._reset_round()
        if self.autocast_dtype is None:
            return self.module(*args, **kw)
        dev = next((t.device.type for t in args if isinstance(t, torch.Tensor)), "cpu")
        with torch.autocast(dev, dtype=self.autocast_dtype, enabled=dev == "cuda"):
            out = self.module(*args, **kw)
        return _to_fp32(out)

    @contextlib.contextmanager
    def no_sync(self):
        old = self._sync
        self._sync = False
        try:
            yield
        finally:
            self._sync = old

    def zero_grad(self, set_to_none: bool = False):
        if self.flat is not None:
            self.flat.zero_()
            self.flat.attach()

    def state_dict(self, *a, **k):
        return self.module.state_dict(*a, **k)

    def load_state_dict(self, sd, strict: bool = True):
        return self.module.load_state_dict(sd, strict=strict)

    @property
    def grad_buffer(self) -> Optional[torch.Tensor]:
        return self.flat.buffer if self.flat is not None else None


def _to_fp32(out):
    if isinstance(out, torch.Tensor):
        return out.float() if out.is_floating_point() else out
    if isinstance(out, (list, tuple)):
        return type(out)(_to_fp32(o) for o in out)
    if isinstance(out, dict):
        return {k: _to_fp32(v) for k, v in out.items()}
    return out


def unwrap(model: nn.Module) -> nn.Module:
    """``model.module`` for wrapped models (the reference's ``ddp_model.module.state_dict()``)."""
    while hasattr(model, "module") and isinstance(model.module, nn.Module):
        model = model.module
    return model
