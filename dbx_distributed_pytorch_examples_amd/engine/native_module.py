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
  the program is compiled for a given batch x image size, or lazily for the first training
  batch (``Accelerator.prepare`` / ``ray.prepare_model`` wrap supported ResNets that way by
  default); batches of another size (a short final batch) run through the plain
  torch module on the same parameters (correct, not accelerated); at world size > 1 their
  gradients are all-reduced too, at the end of that backward (queued autograd callback), so the
  replicas never diverge on a short batch;
* gradients: a backward sets ``p.grad`` (or adds into a ``p.grad`` the caller owns); there is no
  accumulation across two backwards into the same view (call ``zero_grad`` between steps, the
  usual loop);
* world size > 1: rank 0's parameters and BN buffers are broadcast at construction (DDP's
  constructor semantics); the flat gradient is all-reduced (averaged) per
  backward segment on a comm stream while the remaining segments' backward runs (the segment
  boundaries NativeTrainer uses: head+layer4 | layer3 | layer2 | layer1 | stem), so most of the
  all-reduce hides under the backward; do not wrap the result in DDP as well
  (``frontends.accelerate`` knows this). A ``torch.nn.parallel.DistributedDataParallel`` wrap (what
  the real HF ``Accelerator.prepare`` does at world > 1) is neutralised at the first forward: its
  reducer never sees this module's gradients (they are set, not accumulated by autograd), so it is
  switched to ``no_sync`` permanently and stops broadcasting buffers -- the module's own overlapped
  all-reduce is the one gradient synchronisation;
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

from .program import ResNetProgram, supports, release_dead_graphs


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
    def __init__(self, model: nn.Module, batch: Optional[int], image_hw: Optional[Tuple[int, int]],
                 device: torch.device, process_group=None):
        """``batch`` / ``image_hw`` None: compile lazily, for the shape of the first training batch
        (``ray.prepare_model`` / ``Accelerator.prepare`` see no loader shape). The Parameter objects
        of ``model`` stay the same (re-pointed at the flat master), so an optimizer created before
        or after wrapping steps the live weights either way."""
        super().__init__()
        if not supports(model):
            raise TypeError(f"native_module: {type(model).__name__} is not a supported ResNet")
        self.model = model.to(device)
        self.dev = device
        self.pg = process_group
        self.prog = None
        from ..engine_config import EngineConfig
        self.use_graphs = device.type == "cuda" and EngineConfig.current().native_module_graphs
        self._graphs = {}  # "fwd_train" / "fwd_eval" / "bwd*" -> CUDAGraph
        self._calls = {}
        # autograd needs one leaf that requires grad to route the loss back into _NativeFn
        self._anchor = nn.Parameter(torch.zeros((), device=device), requires_grad=True)
        self._grad_views = []
        self.world = dist.get_world_size(process_group) if (dist.is_available() and dist.is_initialized()) else 1
        self._comm = None
        self._fallback_active = False
        self._sync_queued = False
        if self.world > 1:
            self._init_distributed()
        # the torch-module path (another batch shape) produces weight gradients in the conv backward's
        # layout (contiguous); the parameters are channels-last views of the program's KRSC master, so
        # autograd's accumulation would otherwise break the gradient layout contract (a copy per
        # gradient, and a .grad that is no longer a view of the flat gradient buffer)
        for prm in self.model.parameters():
            if prm.dim() == 4 and prm.requires_grad:
                prm.register_hook(_grad_to_param_layout(prm))
        if batch:
            self._build(int(batch), tuple(image_hw))

    def _build(self, batch: int, image_hw: Tuple[int, int]) -> None:
        """Compile the program (parameters / BN buffers move into its flat buffers, same objects)."""
        self.prog = p = ResNetProgram(self.model, batch, image_hw, self.dev)
        p.build_backward()
        self._grad_views = []
        for prm in self.model.parameters():
            off = (prm.data_ptr() - p.master.data_ptr()) // 4
            n = prm.numel()
            g = p.grad[off:off + n]
            gv = g.view(prm.shape[0], prm.shape[2], prm.shape[3], prm.shape[1]).permute(0, 3, 1, 2) \
                if prm.dim() == 4 else g.view(prm.shape)
            self._grad_views.append((prm, gv))
        if self.world > 1:
            self._seg_ranges = []
            for rs in p.segment_param_ranges():
                self._seg_ranges.append((min(r[1] for r in rs), max(r[1] + (r[2] + 15) // 16 * 16 for r in rs))
                                        if rs else None)
            if p.dev.type == "cuda":
                self._comm = torch.cuda.Stream(device=p.dev, priority=-1)
                # next to the comm stream the wgrad side stream costs more than it overlaps
                # (NativeTrainer, profiles/r2s2_multirank/): weight gradients run on the main stream
                p.overlap_wgrad = False
                p.side_batch = p.side_block = False

    # ------------------------------------------------------------------------------
    def _init_distributed(self):
        """DDP-constructor semantics (rank 0's weights and BN buffers everywhere) and the
        short-batch fallback's gradient sync."""
        from ..parallel.dist import host_sync_for_gloo
        pg = self.pg
        src = 0 if pg is None else dist.get_global_rank(pg, 0)
        with torch.no_grad():
            for t in list(self.model.parameters()) + list(self.model.buffers()):
                host_sync_for_gloo(t, pg)
                dist.broadcast(t.data, src, group=pg)
        for prm in self.model.parameters():
            if prm.requires_grad:
                prm.register_post_accumulate_grad_hook(self._fallback_hook)

    def _allreduce_range(self, lo: int, hi: int):
        from ..parallel.dist import host_sync_for_gloo
        g = self.prog.grad[lo:hi]
        host_sync_for_gloo(g, self.pg)
        dist.all_reduce(g, group=self.pg)

    def _fallback_hook(self, prm):
        # the torch-module path (batch of another size) at world > 1: all-reduce its gradients once
        # the whole backward has accumulated them (what DDP would have done)
        if self._fallback_active and not self._sync_queued:
            self._sync_queued = True
            torch.autograd.Variable._execution_engine.queue_callback(self._fallback_allreduce)

    def _fallback_allreduce(self):
        from ..parallel.dist import host_sync_for_gloo
        self._sync_queued = False
        self._fallback_active = False
        grads = [prm.grad for prm in self.model.parameters() if prm.requires_grad and prm.grad is not None]
        if not grads:
            return
        flat = torch._utils._flatten_dense_tensors([g.contiguous() for g in grads])
        host_sync_for_gloo(flat, self.pg)
        dist.all_reduce(flat, group=self.pg)
        flat.div_(self.world)
        for g, r in zip(grads, torch._utils._unflatten_dense_tensors(flat, grads)):
            g.copy_(r)

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
    def _neutralize_outer_ddp(self) -> None:
        """Inside a torch DDP wrapper's forward: make that wrapper inert (see the module docstring)."""
        from torch.nn.parallel import DistributedDataParallel as TorchDDP
        get = getattr(TorchDDP, "_get_active_ddp_module", None)
        d = get() if get is not None else None
        if d is None or d.module is not self or getattr(d, "_dbx_inert", False):
            return
        # _post_forward (after this forward returns) then skips reducer.prepare_for_backward, and
        # every later forward skips the reducer and the buffer broadcast
        d.require_backward_grad_sync = False
        d.require_forward_param_sync = False
        d.broadcast_buffers = False
        d._dbx_inert = True
        import warnings
        warnings.warn("native_module wrapped in torch DistributedDataParallel: the wrapper is made inert; the "
                      "native module all-reduces its own gradients (overlapped with its backward)", stacklevel=3)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        self._neutralize_outer_ddp()
        if (self.prog is None and x.dim() == 4 and x.is_cuda and self.training and torch.is_grad_enabled()
                and x.shape[1] == self.model.conv1.in_channels):
            self._build(x.shape[0], tuple(x.shape[2:]))  # lazy: the first training batch's shape
        p = self.prog
        if (p is None or x.dim() != 4 or x.shape[0] != p.N or tuple(x.shape[2:]) != (p.H, p.W)
                or x.shape[1] != p.in_ch):
            # another batch size / resolution: the torch module on the same parameters (gradients
            # all-reduced after its backward at world > 1, see _fallback_hook)
            self._fallback_active = self.world > 1 and torch.is_grad_enabled() and self.training
            return self.model(x)
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
            release_dead_graphs(self.prog.dev)
            g = torch.cuda.CUDAGraph()
            mode = "thread_local" if (dist.is_available() and dist.is_initialized()) else "global"
            with torch.cuda.graph(g, capture_error_mode=mode):
                fn()
            torch.cuda.synchronize(self.prog.dev)
            self._graphs[key] = g
        g.replay()

    def _fwd_body(self):
        p = self.prog
        p.prepare_weights(step=p.training)  # (training: + statistics zeroing, num_batches_tracked)
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
        if self.world == 1:
            self._run("bwd", p.backward)
        else:
            # one graph per backward segment; each segment's gradient range is all-reduced on the
            # comm stream while the next segment's backward runs (the reference's DDP overlap, M3)
            cur = torch.cuda.current_stream(p.dev) if self._comm is not None else None
            for k, (_, fn) in enumerate(p.backward_segments()):
                self._run(f"bwd{k}", fn)
                rg = self._seg_ranges[k]
                if rg is None:
                    continue
                if cur is None:
                    self._allreduce_range(*rg)
                    continue
                self._comm.wait_stream(cur)
                with torch.cuda.stream(self._comm):
                    self._allreduce_range(*rg)
            if cur is not None:
                cur.wait_stream(self._comm)
            p.grad.div_(self.world)
        for prm, gv in self._grad_views:
            if not prm.requires_grad:
                continue
            if prm.grad is None or prm.grad is gv:
                prm.grad = gv
            else:
                prm.grad.add_(gv)


def _grad_to_param_layout(prm: torch.Tensor):
    def hook(g: torch.Tensor) -> torch.Tensor:
        cl = torch.channels_last
        if prm.is_contiguous(memory_format=cl) and not prm.is_contiguous() and not g.is_contiguous(memory_format=cl):
            return g.contiguous(memory_format=cl)
        return g
    return hook


def native_module(model: nn.Module, batch: Optional[int] = None, image_hw: Optional[Tuple[int, int]] = (224, 224),
                  device: Optional[torch.device] = None, process_group=None) -> NativeResNet:
    """Wrap a supported ResNet (torchvision-layout ResNet-18/34/50/..., the CIFAR-stem ResNet-18)
    for a fixed ``batch`` x ``image_hw`` (``batch=None``: for the first training batch's shape);
    see the module docstring."""
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    return NativeResNet(model, batch, image_hw, device, process_group)
