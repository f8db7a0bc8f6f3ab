"""Frozen-backbone training on the native program: the reference's dominant workload.

Every TorchDistributor / DeepSpeed ResNet notebook trains only a new head on an ImageNet-pretrained
backbone (`models.FrozenBackboneClassifier`, SURVEY C18: `02_cifar…:141-159`, `03_tiny…:125-143`,
`03_1k…:121-139`): ``resnet.fc = Sequential(Dropout(0.5), Linear(in, C))`` with every backbone
parameter frozen. Running that through autograd wastes the backbone's activation memory and
BN-training passes. Here the backbone runs as the native NHWC program in inference mode (BN
folded to per-channel scale/shift from the running statistics, no statistics, no activations kept
for backward) up to the pooled features, and only the head — dropout + linear, ≤ 2 M parameters —
is trained with autograd, its gradients all-reduced over the ranks by the flat-bucket DDP.

The backbone forward (~150 kernels for ResNet-50; launch-bound at the reference's small batches,
e.g. ResNet-18 on 32x32 CIFAR images) is captured as one HIP graph after two eager warm-up
calls and replayed from then on: inputs are copied into the program's static buffers outside
the graph, the features come back in the program's static ``pooled`` buffer. No collective runs
inside it, so the same graph serves every world size. At world size 1 with Adam / AdamW (every
frozen-backbone notebook of the reference uses Adam) the WHOLE step is one graph instead: backbone,
head forward / backward (autograd, captured), a capturable optimizer whose learning rate lives in a
device tensor (``set_lr`` follows on every replay) and the device-side metrics. A short final
batch runs eagerly.
"""
from __future__ import annotations

from typing import Optional, Tuple

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..config import OptimizerConfig
from ..models.wrappers import FrozenBackboneClassifier
from ..parallel.ddp import DistributedDataParallel
from ..utils import debug as _debug
from .autograd_trainer import build_torch_optimizer
from .program import ResNetProgram


def _backbone_proxy(model: FrozenBackboneClassifier) -> nn.Module:
    """The backbone with a plain Linear as ``fc`` (the program needs one; unused for features)."""
    r = model.resnet
    proxy = nn.Module.__new__(type(r))
    proxy.__dict__ = dict(r.__dict__)
    proxy._modules = dict(r._modules)
    proxy._modules["fc"] = nn.Linear(r.fc[-1].in_features, 8)
    return proxy


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
        self.ddp = DistributedDataParallel(self.head, bucket_cap_mb=bucket_cap_mb, allreduce_dtype=allreduce_dtype)
        self.smoothing = label_smoothing
        self.metrics = torch.zeros(2, device=device)  # loss sum, correct (device-side, no host sync)
        self.use_graphs = (use_graphs and device.type == "cuda" and not _debug.enabled()
                           and os.environ.get("DBX_FROZEN_GRAPHS", "1") != "0")
        self._graph = None
        self._feats = None
        self._warm = 0
        params = [p for p in self.head.parameters() if p.requires_grad]
        # whole-step graph: pays off where the step is launch-bound (measured on one MI355X,
        # profiles/r2s5_frozen/: ResNet-18 CIFAR b256 530k vs 455k img/s with the backbone-only graph);
        # for larger inputs the capturable optimizer costs a little more than the head launches it
        # hides (ResNet-50 64x64 / 224x224: -2..-3 %). DBX_FROZEN_FULL_GRAPH=1 / 0 forces it.
        mode = os.environ.get("DBX_FROZEN_FULL_GRAPH", "auto")
        small = batch * image_hw[0] * image_hw[1] <= 256 * 32 * 32
        self.full_graph = (self.use_graphs and self.ddp.world == 1 and optim.name in ("adam", "adamw")
                           and (mode == "1" or (mode == "auto" and small)))
        self.lr_t = None
        if self.full_graph:
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
            torch.cuda.synchronize(self.dev)
            s = torch.cuda.Stream(device=self.dev)
            s.wait_stream(torch.cuda.current_stream(self.dev))
            g = torch.cuda.CUDAGraph()
            import torch.distributed as dist
            # thread-local capture next to a process group's watchdog thread (see NativeTrainer._capture)
            mode = "thread_local" if (dist.is_available() and dist.is_initialized()) else "global"
            with torch.cuda.stream(s):
                with torch.cuda.graph(g, stream=s, capture_error_mode=mode):
                    self._feats = self._run_backbone()
            torch.cuda.current_stream(self.dev).wait_stream(s)
            self._graph = g
        self._graph.replay()
        return self._feats

    def set_lr(self, lr: float):
        if self.lr_t is not None:
            self.lr_t.fill_(float(lr))  # the captured optimizer reads it on every replay
            return
        for g in self.opt.param_groups:
            g["lr"] = float(lr)

    def _features(self, images_u8, labels, boxes, flips) -> torch.Tensor:
        self._stage_inputs(images_u8, boxes, flips)
        return self._backbone()[:images_u8.shape[0]]

    def step(self, images_u8, labels, boxes=None, flips=None):
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
                        self._head_step(self._backbone_eager().float(), self.lab)
                    cur.wait_stream(s)
                    return
                torch.cuda.synchronize(self.dev)
                g = torch.cuda.CUDAGraph()
                # thread-local whenever a process group (and its watchdog thread) exists, even at world 1
                mode = "thread_local" if (dist.is_available() and dist.is_initialized()) else "global"
                with torch.cuda.graph(g, capture_error_mode=mode):
                    self._head_step(self._backbone_eager().float(), self.lab)
                torch.cuda.synchronize(self.dev)
                self._sgraph = g
            self._sgraph.replay()
            return
        feats = self._features(images_u8, labels, boxes, flips).float()
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
        feats = self._features(images_u8, labels, boxes, None).float()
        self.head.eval()
        out = self.head(feats)
        self.head.train()
        return out

    def read_metrics(self, reset: bool = True):
        m = self.metrics.tolist()
        if reset:
            self.metrics.zero_()
        return m[0], m[1]
