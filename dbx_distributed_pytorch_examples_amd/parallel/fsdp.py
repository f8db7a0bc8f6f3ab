"""ZeRO-3: parameter-sharded data parallelism (+ optional CPU offload) for any ``nn.Module``.

The reference ships DeepSpeed ``zero_3`` and ``zero_3_offload`` dicts
(`/root/reference/02_deepspeed/deepspeed_config.py:74-84`, `:87-105`: ``stage: 3``,
``offload_optimizer``/``offload_param: {device: cpu, pin_memory: true}``) but never hands them to
DeepSpeed. This module makes them real on the autograd engine.

Design (one process per GPU, RCCL collectives on the compute stream):

* the model is cut into **units** (each residual block, each other container child of the root;
  leaf parameters of the root form one root unit). A unit's parameters are flattened, trainable
  first, padded to ``world * per`` and every rank keeps only its contiguous ``per``-element fp32
  shard (plus the optimizer moments of that shard);
* a unit's full flat buffer is materialised by one ``all_gather_into_tensor`` in a forward
  pre-hook and its storage is released (``resize_(0)``) after the unit's forward; a hook on the
  unit's outputs re-gathers it when their gradient arrives, i.e. right before the unit's
  backward. Parameters are views of that one storage, so tensors autograd saved stay valid across
  the release / re-gather (same storage object, new allocation);
* when the last trainable parameter of a unit has accumulated its gradient, the unit's gradients
  are packed into one padded flat buffer and ``reduce_scatter``-ed (pre-divided by the world size)
  into the rank's gradient shard, and the full parameters are released again — so at any moment
  only the units currently executing are materialised;
* the optimizer step runs the fused HIP SGD/Adam kernels over each unit's trainable shard region;
  with ``offload_optimizer`` the fp32 master shard and the moments live in pinned host memory and
  the step runs on the CPU (gradient shard D2H, updated shard H2D); with ``offload_param`` no
  persistent device copy of the shard is kept either (it is uploaded at each gather).

DeepSpeed ``stage3_*`` knobs: ``persistence_threshold`` keeps units with fewer parameter elements
than it replicated (gathered once, re-gathered after each optimizer step, never released:
DeepSpeed's ``stage3_param_persistence_threshold``, at unit rather than parameter granularity);
``prefetch_elems`` lets a unit's forward pre-hook issue the asynchronous all-gathers of the units
after it, up to that many elements ahead (``stage3_prefetch_bucket_size``), so their transfer
overlaps the current unit's compute.

Buffers (BatchNorm running statistics) stay replicated, broadcast from rank 0 at construction, as
DeepSpeed and torch FSDP do. ``state_dict()`` / ``load_state_dict()`` on the wrapped module work
on full tensors (hooks gather first; every rank must call them, as with any collective).
"""
from __future__ import annotations

import contextlib
from typing import Dict, List, Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from ..ops import kernels as K
from .dist import host_sync_for_gloo


def _has_params(m: nn.Module) -> bool:
    return any(True for _ in m.parameters())


def _has_seq(m: nn.Module) -> bool:
    return any(isinstance(c, (nn.Sequential, nn.ModuleList)) for c in m.children())


def _default_units(model: nn.Module) -> List[nn.Module]:
    """Residual blocks / container children (Sequential and ModuleList expanded; wrappers around a
    backbone, e.g. ``ComposerResNet50.model``, recursed into). Leaf children stay in the root unit."""
    units = []
    for child in model.children():
        if not _has_params(child):
            continue
        if isinstance(child, (nn.Sequential, nn.ModuleList)):
            for sub in child:
                if _has_params(sub):
                    units.append(sub)
        elif _has_seq(child):
            units.extend(_default_units(child))
        elif any(True for _ in child.children()):
            units.append(child)
    return units


def _tensors(out):
    if isinstance(out, torch.Tensor):
        yield out
    elif isinstance(out, (list, tuple)):
        for o in out:
            yield from _tensors(o)
    elif isinstance(out, dict):
        for o in out.values():
            yield from _tensors(o)


class _Unit:
    def __init__(self, owner: "ShardedDataParallel", name: str, params: List[nn.Parameter], reshard: bool,
                 persistent: bool = False):
        self.owner, self.name, self.reshard = owner, name, reshard
        self.persistent = persistent
        self.work = None  # in-flight asynchronous all-gather (prefetch)
        params = [p for p in params if p.requires_grad] + [p for p in params if not p.requires_grad]
        self.params = params
        self.trainable = [p for p in params if p.requires_grad]
        self.n_train = sum(p.numel() for p in self.trainable)
        self.n = sum(p.numel() for p in params)
        w, r = owner.world, owner.rank
        self.per = max(16, ((self.n + w - 1) // w + 15) // 16 * 16)
        self.padded = self.per * w
        dev = owner.device
        self.full = torch.zeros(self.padded, device=dev)
        off = 0
        with torch.no_grad():
            for p in params:
                self.full[off:off + p.numel()].copy_(p.detach().reshape(-1))
                off += p.numel()
        if w > 1:  # replicas start from rank 0's initialisation (DDP semantics)
            host_sync_for_gloo(self.full)
            dist.broadcast(self.full, 0, group=owner.pg)
        off = 0
        for p in params:
            p.data = self.full[off:off + p.numel()].view(p.shape)
            off += p.numel()
        # trainable elements of this rank's shard: [0, k) (trainable params come first)
        self.k = max(0, min(self.per, self.n_train - r * self.per))
        host = owner.offload_optimizer
        shard = self.full[r * self.per:(r + 1) * self.per].detach().clone()
        self.master = shard.cpu().pin_memory() if host and dev.type == "cuda" else (shard.cpu() if host else shard)
        self.dev_shard = None if owner.offload_param else (shard if not host else shard.clone())
        sdev = self.master.device
        self.m = torch.zeros(self.per, device=sdev)
        self.v = torch.zeros(self.per, device=sdev) if owner.o.name in ("adam", "adamw") else None
        self.gshard = torch.zeros(self.per, device=dev)
        self.gathered = True
        self.pinned = False
        self.ready = 0
        self.release(force=True)
        if persistent:
            self.gather()

    # -- parameter materialisation -----------------------------------------------------------
    def wait(self):
        if self.work is not None:
            self.work.wait()
            self.work = None
            self._src = None

    def gather(self, async_op: bool = False):
        if self.gathered:
            if not async_op:
                self.wait()
            return
        o = self.owner
        st = self.full.untyped_storage()
        st.resize_(self.padded * self.full.element_size())
        src = self.dev_shard
        if src is None:  # offload_param: upload the host shard
            src = self.master.to(o.device, non_blocking=True)
        if o.world > 1:
            host_sync_for_gloo(src)
            w = dist.all_gather_into_tensor(self.full, src, group=o.pg, async_op=async_op)
            if async_op:
                self.work, self._src = w, src  # the source stays alive until the gather completes
        else:
            self.full.copy_(src)
        self.gathered = True

    def release(self, force: bool = False):
        if not self.gathered or ((self.pinned or self.persistent) and not force):
            return
        self.wait()
        # queued kernels may still read the storage; the caching allocator orders its reuse on this
        # stream, the only one that touches it
        self.full.untyped_storage().resize_(0)
        self.gathered = False

    # -- gradients ---------------------------------------------------------------------------
    def on_grad(self):
        self.ready += 1
        if self.ready == len(self.trainable):
            if self.owner._no_sync:  # gradient accumulation: grads stay in p.grad until the last micro-step
                self.ready = 0
            else:
                self.reduce()

    def reduce(self):
        o = self.owner
        self.ready = 0
        if not self.trainable:
            return
        flat = torch.zeros(self.padded, device=o.device)
        off = 0
        for p in self.trainable:
            if p.grad is not None:
                flat[off:off + p.numel()].copy_(p.grad.reshape(-1))
            p.grad = None
            off += p.numel()
        flat.mul_(1.0 / o.world)
        if o.world > 1:
            host_sync_for_gloo(flat, o.pg)
            part = torch.empty(self.per, device=o.device)
            try:
                dist.reduce_scatter_tensor(part, flat, group=o.pg)
            except (RuntimeError, NotImplementedError, AttributeError):
                dist.all_reduce(flat, group=o.pg)
                part = flat[o.rank * self.per:(o.rank + 1) * self.per]
            self.gshard.add_(part)
        else:
            self.gshard.add_(flat)
        if len(self.trainable) == len(self.params):  # frozen params may still be needed by backward
            self.release()


class ShardedDataParallel(nn.Module):
    """ZeRO stage 3 wrapper. ``optim``: fields name, lr, momentum, nesterov, weight_decay, betas,
    eps, grad_clip (the TrainConfig ``OptimConfig``)."""

    def __init__(self, module: nn.Module, optim, process_group=None, units: Optional[List[nn.Module]] = None,
                 offload_optimizer: bool = False, offload_param: bool = False, reshard_after_forward: bool = True,
                 persistence_threshold: int = 0, prefetch_elems: int = 0):
        super().__init__()
        self.prefetch_elems = int(prefetch_elems)
        if optim.name not in ("sgd", "adam", "adamw"):
            raise ValueError(f"ZeRO-3 supports sgd / adam / adamw, not {optim.name!r}")
        self.module = module
        self.o = optim
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_available() and dist.is_initialized() else 1
        self.rank = dist.get_rank(process_group) if self.world > 1 else 0
        self.device = next(module.parameters()).device
        self.offload_optimizer = offload_optimizer or offload_param
        self.offload_param = offload_param
        self._no_sync = False
        self.step_count = 0
        if self.world > 1:
            for b in module.buffers():
                host_sync_for_gloo(b)
                dist.broadcast(b, 0, group=self.pg)
        units = _default_units(module) if units is None else units
        names = {id(m): n for n, m in module.named_modules()}
        owned = set()
        self.units: List[_Unit] = []
        for m in units:
            ps = [p for p in m.parameters() if id(p) not in owned]
            owned.update(id(p) for p in ps)
            if ps:
                persistent = sum(p.numel() for p in ps) < persistence_threshold
                u = _Unit(self, names.get(id(m), "?"), ps, reshard_after_forward, persistent)
                self.units.append(u)
                self._hook_unit(m, u)
        rest = [p for p in module.parameters() if id(p) not in owned]
        self.root = _Unit(self, "<root>", rest, False) if rest else None
        module.register_forward_pre_hook(self._root_pre)
        module.register_forward_hook(self._root_post)
        if self.root is not None:
            for p in self.root.trainable:
                p.register_post_accumulate_grad_hook(lambda _p, u=self.root: u.on_grad())
        module._register_state_dict_hook(self._sd_post)
        module.register_state_dict_pre_hook(lambda *a, **k: self.gather_full_params())
        module._register_load_state_dict_pre_hook(lambda *a, **k: self.gather_full_params())
        module.register_load_state_dict_post_hook(lambda *a, **k: self._reshard_from_full())

    # -- hooks -------------------------------------------------------------------------------
    def _hook_unit(self, m: nn.Module, u: _Unit):
        def pre(_m, _inp):
            u.gather()
            self._prefetch_after(u)

        def post(_m, _inp, out):
            if torch.is_grad_enabled():
                for t in _tensors(out):
                    if t.requires_grad:
                        t.register_hook(lambda g: (u.gather(), g)[1])
            if u.reshard:
                u.release()
        m.register_forward_pre_hook(pre)
        m.register_forward_hook(post)
        for p in u.trainable:
            p.register_post_accumulate_grad_hook(lambda _p: u.on_grad())

    def _prefetch_after(self, u: _Unit):
        """Issue the asynchronous all-gathers of the units after ``u`` (forward order) within the
        prefetch budget; their own pre-hooks wait for them."""
        if self.prefetch_elems <= 0 or self.world == 1:
            return
        budget = self.prefetch_elems
        i = self.units.index(u)
        for v in self.units[i + 1:]:
            if v.n > budget:
                break
            budget -= v.n
            v.gather(async_op=True)

    def _root_pre(self, _m, _inp):
        if torch.is_grad_enabled():
            for u in self._all():
                u.pinned = False
        if self.root is not None:
            self.root.gather()

    def _root_post(self, _m, _inp, _out):
        if self.root is not None and not torch.is_grad_enabled():
            self.root.release()

    def _all(self) -> List[_Unit]:
        return self.units + ([self.root] if self.root is not None else [])

    def forward(self, *args, **kw):
        return self.module(*args, **kw)

    @contextlib.contextmanager
    def no_sync(self):
        self._no_sync = True
        try:
            yield
        finally:
            self._no_sync = False

    # -- full-parameter views (checkpointing / evaluation) -----------------------------------
    @torch.no_grad()
    def gather_full_params(self):
        """Materialise every unit and keep it until the next training forward (all ranks)."""
        for u in self._all():
            u.gather()
            u.pinned = True

    def _sd_post(self, _m, sd, prefix, _local):
        for k, v in list(sd.items()):
            sd[k] = v.detach().clone()
        return sd

    @torch.no_grad()
    def _reshard_from_full(self):
        for u in self._all():
            lo = self.rank * u.per
            shard = u.full[lo:lo + u.per]
            u.master.copy_(shard)
            if u.dev_shard is not None:
                u.dev_shard.copy_(shard)

    # -- gradient sync / optimizer -----------------------------------------------------------
    def finish_gradient_sync(self):
        """Reduce units whose gradients did not all arrive (unused params), in unit order."""
        for u in self._all():
            if u.trainable and any(p.grad is not None for p in u.trainable):
                u.reduce()
            u.ready = 0
            if u.reshard or u is self.root:
                u.release()

    def zero_grad(self):
        for u in self._all():
            u.gshard.zero_()
            for p in u.trainable:
                p.grad = None

    @torch.no_grad()
    def optimizer_step(self, lr: Optional[float] = None):
        o = self.o
        self.step_count += 1
        lr = o.lr if lr is None else lr
        units = [u for u in self._all() if u.k > 0]
        coef = None
        if getattr(o, "grad_clip", 0.0):
            local = torch.zeros((), device=self.device)
            for u in units:
                local += u.gshard[:u.k].pow(2).sum()
            if self.world > 1:
                host_sync_for_gloo(local, self.pg)
                dist.all_reduce(local, group=self.pg)
            coef = torch.clamp(o.grad_clip / (local.sqrt() + 1e-6), max=1.0)
        for u in units:
            g = u.gshard[:u.k]
            if coef is not None:
                g.mul_(coef)
            if u.master.device != g.device:
                g = g.to(u.master.device)
            p, m = u.master[:u.k], u.m[:u.k]
            if o.name == "sgd":
                K.sgd_step(p, g, m, None, lr=lr, momentum=o.momentum, dampening=getattr(o, "dampening", 0.0),
                           weight_decay=o.weight_decay, nesterov=o.nesterov, first=False)
            else:
                K.adam_step(p, g, m, u.v[:u.k], None, lr=lr, beta1=o.betas[0], beta2=o.betas[1], eps=o.eps,
                            weight_decay=o.weight_decay, decoupled=(o.name == "adamw"), step=self.step_count)
            if u.dev_shard is not None and u.dev_shard is not u.master:
                u.dev_shard[:u.k].copy_(p, non_blocking=True)
        for u in self._all():  # materialised copies are stale now (other ranks updated their shards)
            u.pinned = False
            u.release(force=True)
            if u.persistent:
                u.gather()

    def optim_state_dict(self) -> Dict:
        return {"stage": 3, "step": self.step_count, "rank": self.rank, "world": self.world,
                "m": [u.m.cpu() for u in self._all()],
                "v": [None if u.v is None else u.v.cpu() for u in self._all()],
                "master": [u.master.cpu() for u in self._all()]}

    def load_optim_state_dict(self, sd: Dict):
        if sd["world"] != self.world:
            raise ValueError("ZeRO-3 state was saved with a different world size")
        self.step_count = int(sd["step"])
        for u, m, v, p in zip(self._all(), sd["m"], sd["v"], sd["master"]):
            u.m.copy_(m)
            if u.v is not None and v is not None:
                u.v.copy_(v)
            u.master.copy_(p)
            if u.dev_shard is not None and u.dev_shard is not u.master:
                u.dev_shard.copy_(p)
            u.pinned = False
            u.release(force=True)
            if u.persistent:
                u.gather()

    def materialised_bytes(self) -> int:
        return sum(u.full.untyped_storage().nbytes() for u in self._all())
