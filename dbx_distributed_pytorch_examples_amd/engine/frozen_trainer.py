"""Frozen-backbone training on the native program: the reference's dominant workload.

Every TorchDistributor / DeepSpeed ResNet notebook trains only a new head on an ImageNet-pretrained
backbone (`models.FrozenBackboneClassifier`, SURVEY C18: `02_cifar…:141-159`, `03_tiny…:125-143`,
`03_1k…:121-139`): ``resnet.fc = Sequential(Dropout(0.5), Linear(in, C))`` with every backbone
parameter frozen. Running that through autograd wastes the backbone's activation memory and
BN-training passes. Here the backbone runs as the native NHWC program in inference mode (BN
folded to per-channel scale/shift from the running statistics, no statistics, no activations kept
for backward) up to the pooled features, and only the head — dropout + linear, ≤ 2 M parameters —
is trained, by :class:`NativeHead` on the HIP kernels: the fc GEMMs on MFMA with the bias and a
Philox dropout mask fused into the operand loads (the weight gradient regenerates the forward's
mask from (seed, step) instead of storing it), the fused softmax-CE, the bias-gradient column sum
and the fused Adam / SGD over the head's flat fp32 master (engine field ``frozen_native_head=0``: the
autograd head with the flat-bucket DDP). At world > 1 the head's flat gradient is all-reduced once.

The backbone forward (~150 kernels for ResNet-50; launch-bound at the reference's small batches,
e.g. ResNet-18 on 32x32 CIFAR images) is captured as one HIP graph after two eager warm-up
calls and replayed from then on: inputs are copied into the program's static buffers outside
the graph, the features come back in the program's static ``pooled`` buffer. No collective runs
inside it, so the same graph serves every world size. At world size 1 with Adam / AdamW (every
frozen-backbone notebook of the reference uses Adam) the WHOLE step is one graph instead: backbone,
head forward / backward, the optimizer reading its learning rate / bias corrections from a device
tensor (``set_lr`` follows on every replay) and the device-side metrics. A short final batch runs
eagerly.
"""
from __future__ import annotations

from typing import Optional, Tuple

import os

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

from ..config import OptimizerConfig
from ..models.wrappers import FrozenBackboneClassifier
from ..parallel.ddp import DistributedDataParallel
from ..utils import debug as _debug
from .autograd_trainer import build_torch_optimizer
from .hyper import DeviceHyper
from .program import ResNetProgram, release_dead_graphs
from ..engine_config import EngineConfig


def _backbone_proxy(model: FrozenBackboneClassifier) -> nn.Module:
    """The backbone with a plain Linear as ``fc`` (the program needs one; unused for features)."""
    r = model.resnet
    proxy = nn.Module.__new__(type(r))
    proxy.__dict__ = dict(r.__dict__)
    proxy._modules = dict(r._modules)
    proxy._modules["fc"] = nn.Linear(r.fc[-1].in_features, 8)
    return proxy


class NativeHead:
    """``[Dropout(p) ->] Linear(F, C)`` trained on the native kernels (see the module docstring).
    The module's Parameter objects are re-pointed at the head's flat fp32 master (``.data``)."""

    def __init__(self, head: nn.Module, batch: int, device: torch.device, optim: OptimizerConfig,
                 label_smoothing: float = 0.0, seed: int = 0):
        from ..ops import kernels as K
        self.K = K
        lins = [m for m in head.modules() if isinstance(m, nn.Linear)]
        if len(lins) != 1 or any(not isinstance(m, (nn.Linear, nn.Dropout, nn.Sequential, nn.Identity))
                                 for m in head.modules()):
            raise TypeError("NativeHead supports [Dropout ->] Linear heads")
        lin = lins[0]
        drops = [m for m in head.modules() if isinstance(m, nn.Dropout)]
        self.p_drop = float(drops[0].p) if drops else 0.0
        self.head, self.lin, self.dev, self.o = head, lin, device, optim
        self.B, self.F, self.C = batch, lin.in_features, lin.out_features
        nW = self.C * self.F
        self.off_b = (nW + 15) // 16 * 16
        n = self.off_b + (self.C + 15) // 16 * 16
        self.master = torch.zeros(n, device=device)
        self.grad = torch.zeros(n, device=device)
        with torch.no_grad():
            self.master[:nW].copy_(lin.weight.detach().reshape(-1))
            if lin.bias is not None:
                self.master[self.off_b:self.off_b + self.C].copy_(lin.bias.detach())
        lin.weight.data = self.master[:nW].view(self.C, self.F)
        if lin.bias is not None:
            lin.bias.data = self.master[self.off_b:self.off_b + self.C]
        self.p16 = self.master.to(torch.bfloat16)  # bf16 compute copy, rewritten by the optimizer kernel
        self.w16 = self.p16[:nW].view(self.C, self.F)
        self.b16 = self.p16[self.off_b:self.off_b + self.C]
        self.gW = self.grad[:nW].view(self.C, self.F)
        self.gb = self.grad[self.off_b:self.off_b + self.C]
        self.m = torch.zeros(n, device=device)
        self.v = torch.zeros(n, device=device) if optim.name in ("adam", "adamw") else None
        self.hyper = torch.zeros(4, device=device)
        self._hyper_dev = DeviceHyper(self.hyper)
        self.step_count = 0
        self.drop_off = torch.zeros(1, device=device, dtype=torch.int32)  # Philox offset: +1 per step (device)
        self.seed = int(seed) * 0x9E3779B97F4A7C15 % (1 << 63) + 12345
        self.logits = torch.empty(batch, self.C, device=device, dtype=torch.bfloat16)
        self.dlogits = torch.empty_like(self.logits)
        self.smoothing = label_smoothing
        self.world = dist.get_world_size() if (dist.is_available() and dist.is_initialized()) else 1

    def _drop(self, which):
        return (which, self.p_drop, self.seed, self.drop_off) if self.p_drop > 0 else None

    def set_hyper(self):
        """host -> device (lr, 1-b1^t, 1-b2^t) for the next step (graph replays read it)."""
        o = self.o
        self.step_count += 1
        t = self.step_count
        vals = [o.lr, 1.0, 1.0, 0.0] if o.name == "sgd" else [o.lr, 1.0 - o.betas[0] ** t, 1.0 - o.betas[1] ** t, 0.0]
        self._hyper_dev.set(vals)

    def fwd_bwd(self, feats: torch.Tensor, labels: torch.Tensor, metrics: torch.Tensor) -> None:
        """feats [n, F] bf16 (n <= batch), labels [n] int64: logits, CE (+ metrics), dW, db."""
        K, n = self.K, feats.shape[0]
        lg, dl = self.logits[:n], self.dlogits[:n]
        K.small_gemm(feats, self.w16, lg, M=n, N=self.C, K=self.F, bias=self.b16, dropout=self._drop("A"))
        K.softmax_ce(lg, labels, dl, None, metrics, smoothing=self.smoothing)
        K.small_gemm(dl, feats, self.gW, ta=True, tb=True, M=self.C, N=self.F, K=n, dropout=self._drop("B"))
        K.colsum(dl, self.gb)

    def allreduce(self) -> None:
        if self.world > 1:
            import torch.distributed as dist
            from ..parallel.dist import host_sync_for_gloo
            host_sync_for_gloo(self.grad, None)
            dist.all_reduce(self.grad)

    def optimizer(self) -> None:
        K, o = self.K, self.o
        gs = 1.0 / self.world
        if o.name == "sgd":
            K.sgd_step(self.master, self.grad, self.m, self.p16, lr=o.lr, momentum=o.momentum,
                       weight_decay=o.weight_decay, nesterov=o.nesterov, first=False, grad_scale=gs, hyper=self.hyper)
        else:
            K.adam_step(self.master, self.grad, self.m, self.v, self.p16, lr=o.lr, beta1=o.betas[0], beta2=o.betas[1],
                        eps=o.eps, weight_decay=o.weight_decay, decoupled=(o.name == "adamw"), step=self.step_count,
                        grad_scale=gs, hyper=self.hyper)
        self.drop_off.add_(1)  # the next step's dropout mask

    @torch.no_grad()
    def eval_logits(self, feats: torch.Tensor) -> torch.Tensor:
        n = feats.shape[0]
        out = torch.empty(n, self.C, device=self.dev, dtype=torch.bfloat16)
        self.K.small_gemm(feats, self.w16, out, M=n, N=self.C, K=self.F, bias=self.b16)
        return out.float()


class FrozenFeatureTrainer:
    """``step(images_u8, labels, boxes, flips)``: native backbone features -> autograd head step."""

    def __init__(self, model: FrozenBackboneClassifier, batch: int, image_hw: Tuple[int, int], device: torch.device,
                 optim: OptimizerConfig, label_smoothing: float = 0.0, src_hw=None, mean=None, std=None,
                 bucket_cap_mb: float = 64.0, allreduce_dtype=torch.float32, use_graphs: bool = True):
        self.full_model = model
        self.dev = device
        self.prog = ResNetProgram(_backbone_proxy(model), batch, image_hw, device, src_hw=src_hw, mean=mean, std=std)
        self.prog.training = False
        self.prog.prepare_weights()  # frozen: converted once
        self.head = model.resnet.fc.to(device)
        self.smoothing = label_smoothing
        self.nhead = None
        eng = EngineConfig.current()
        if eng.frozen_native_head and optim.name in ("sgd", "adam", "adamw"):
            try:
                self.nhead = NativeHead(self.head, batch, device, optim, label_smoothing)
            except TypeError:
                self.nhead = None  # an unsupported head module: the autograd head below
        if self.nhead is not None:
            self.opt_cfg = optim
            self.mom, self.mom2 = self.nhead.m, self.nhead.v  # (native optimizer state for checkpoints)
        self.ddp = DistributedDataParallel(self.head, bucket_cap_mb=bucket_cap_mb, allreduce_dtype=allreduce_dtype,
                                           gradient_sync=self.nhead is None)
        self.metrics = torch.zeros(2, device=device)  # loss sum, correct (device-side, no host sync)
        self.metrics64 = torch.zeros(2, device=device, dtype=torch.float64)  # the same, from the native CE
        self.use_graphs = (use_graphs and device.type == "cuda" and not _debug.enabled()
                           and eng.frozen_graphs)
        self._graph = None
        self._feats = None
        self._warm = 0
        params = [p for p in self.head.parameters() if p.requires_grad]
        # whole-step graph: pays off where the step is launch-bound (measured on one MI355X,
        # profiles/r2s5_frozen/: ResNet-18 CIFAR b256 530k vs 455k img/s with the backbone-only graph);
        # for larger inputs the capturable optimizer costs a little more than the head launches it
        # hides (ResNet-50 64x64 / 224x224: -2..-3 %). frozen_full_graph=1 / 0 forces it.
        mode = eng.frozen_full_graph
        small = batch * image_hw[0] * image_hw[1] <= 256 * 32 * 32
        world = dist.get_world_size() if (dist.is_available() and dist.is_initialized()) else 1
        if self.nhead is not None:  # native head: no autograd / capturable-optimizer cost in the graph
            self.full_graph = self.use_graphs and world == 1 and mode != "0"
        else:
            self.full_graph = (self.use_graphs and world == 1 and optim.name in ("adam", "adamw")
                               and (mode == "1" or (mode == "auto" and small)))
        self.lr_t = None
        if self.nhead is not None:
            self.opt = None
            self.lab = torch.zeros(batch, dtype=torch.int64, device=device)
        elif self.full_graph:
            self.lr_t = torch.tensor(float(optim.lr), device=device)
            cls = torch.optim.Adam if optim.name == "adam" else torch.optim.AdamW
            self.opt = cls(params, lr=self.lr_t, betas=tuple(optim.betas), eps=optim.eps,
                           weight_decay=optim.weight_decay, capturable=True)
            self.lab = torch.zeros(batch, dtype=torch.int64, device=device)  # static labels of the graph
        else:
            self.opt = build_torch_optimizer(params, optim)
        self._sgraph = None
        self._swarm = 0

    def _run_backbone(self) -> torch.Tensor:
        p = self.prog
        p.load_input_u8(None)
        return p.forward(compute_grad=False, metrics=False, features_only=True)

    @torch.no_grad()
    def _backbone(self) -> torch.Tensor:
        if not self.use_graphs:
            return self._run_backbone()
        if self._graph is None:
            if self._warm < 2:  # allocator / library handles settle in eager calls first
                self._warm += 1
                return self._run_backbone()
            release_dead_graphs(self.dev)
            s = torch.cuda.Stream(device=self.dev)
            s.wait_stream(torch.cuda.current_stream(self.dev))
            g = torch.cuda.CUDAGraph()
            # thread-local capture next to a process group's watchdog thread (see NativeTrainer._capture)
            mode = "thread_local" if (dist.is_available() and dist.is_initialized()) else "global"
            with torch.cuda.stream(s):
                with torch.cuda.graph(g, stream=s, capture_error_mode=mode):
                    self._feats = self._run_backbone()
            torch.cuda.current_stream(self.dev).wait_stream(s)
            self._graph = g
        self._graph.replay()
        return self._feats

    @torch.no_grad()
    def params_changed(self) -> None:
        """The model's parameters were rewritten (``load_state_dict`` on resume): refresh the derived
        copies -- the native head's bf16 compute copy (in place: captured graphs read it) and the
        backbone program's converted weights."""
        if self.nhead is not None:
            self.nhead.p16.copy_(self.nhead.master)
        self.prog.prepare_weights()

    @property
    def step_count(self) -> int:
        return self.nhead.step_count if self.nhead is not None else 0

    @step_count.setter
    def step_count(self, v: int) -> None:
        if self.nhead is not None:
            self.nhead.step_count = int(v)

    def set_lr(self, lr: float):
        if self.nhead is not None:
            self.nhead.o.lr = float(lr)  # device-side on the next step (set_hyper)
            return
        if self.lr_t is not None:
            self.lr_t.fill_(float(lr))  # the captured optimizer reads it on every replay
            return
        for g in self.opt.param_groups:
            g["lr"] = float(lr)

    def _features(self, images_u8, labels, boxes, flips) -> torch.Tensor:
        self._stage_inputs(images_u8, boxes, flips)
        return self._backbone()[:images_u8.shape[0]]

    def step(self, images_u8, labels, boxes=None, flips=None):
        if self.nhead is not None:
            self.nhead.set_hyper()
        if self.full_graph and images_u8.shape[0] == self.prog.N:
            self._stage_inputs(images_u8, boxes, flips)
            self.lab.copy_(labels, non_blocking=True)
            if self._sgraph is None:
                cur = torch.cuda.current_stream(self.dev)
                if self._swarm < 2:  # eager warm-up steps on a side stream (optimizer state, autograd)
                    self._swarm += 1
                    s = torch.cuda.Stream(device=self.dev)
                    s.wait_stream(cur)
                    with torch.cuda.stream(s):
                        self._head_step(self._backbone_eager(), self.lab)
                    cur.wait_stream(s)
                    return
                release_dead_graphs(self.dev)
                g = torch.cuda.CUDAGraph()
                # thread-local whenever a process group (and its watchdog thread) exists, even at world 1
                mode = "thread_local" if (dist.is_available() and dist.is_initialized()) else "global"
                with torch.cuda.graph(g, capture_error_mode=mode):
                    self._head_step(self._backbone_eager(), self.lab)
                torch.cuda.synchronize(self.dev)
                self._sgraph = g
            self._sgraph.replay()
            return
        feats = self._features(images_u8, labels, boxes, flips)
        self._head_step(feats, labels.to(self.dev, non_blocking=True))

    @torch.no_grad()
    def _backbone_eager(self) -> torch.Tensor:
        return self._run_backbone()

    def _stage_inputs(self, images_u8, boxes, flips):
        p = self.prog
        n = images_u8.shape[0]
        p.img_u8[:n].copy_(images_u8, non_blocking=True)
        if boxes is not None:
            p.boxes[:n].copy_(boxes, non_blocking=True)
        if flips is not None:
            p.flip[:n].copy_(flips, non_blocking=True)
        else:
            p.flip.zero_()

    def _head_step(self, feats, labels):
        if self.nhead is not None:
            h = self.nhead
            h.fwd_bwd(feats.bfloat16() if feats.dtype != torch.bfloat16 else feats, labels, self.metrics64)
            h.allreduce()
            h.optimizer()
            return
        feats = feats.float()
        self.head.train()
        logits = self.ddp(feats)
        loss = F.cross_entropy(logits, labels, label_smoothing=self.smoothing)
        self.opt.zero_grad(set_to_none=False)
        loss.backward()
        self.ddp.finish_gradient_sync()
        self.opt.step()
        with torch.no_grad():
            self.metrics += torch.stack([loss.detach() * labels.shape[0], (logits.argmax(1) == labels).sum().float()])

    @torch.no_grad()
    def evaluate_batch(self, images_u8, labels, boxes=None) -> torch.Tensor:
        feats = self._features(images_u8, labels, boxes, None)
        if self.nhead is not None:
            return self.nhead.eval_logits(feats.bfloat16())
        feats = feats.float()
        self.head.eval()
        out = self.head(feats)
        self.head.train()
        return out

    def read_metrics(self, reset: bool = True):
        m = self.metrics.tolist()
        m2 = self.metrics64.tolist()
        if reset:
            self.metrics.zero_()
            self.metrics64.zero_()
        return m[0] + m2[0], m[1] + m2[1]
