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
inside it, so the same graph serves every world size.
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
        self.opt = build_torch_optimizer([p for p in self.head.parameters() if p.requires_grad], optim)
        self.smoothing = label_smoothing
        self.metrics = torch.zeros(2, device=device)  # loss sum, correct (device-side, no host sync)
        self.use_graphs = (use_graphs and device.type == "cuda" and not _debug.enabled()
                           and os.environ.get("DBX_FROZEN_GRAPHS", "1") != "0")
        self._graph = None
        self._feats = None
        self._warm = 0

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
        for g in self.opt.param_groups:
            g["lr"] = float(lr)

    def _features(self, images_u8, labels, boxes, flips) -> torch.Tensor:
        p = self.prog
        n = images_u8.shape[0]
        p.img_u8[:n].copy_(images_u8, non_blocking=True)
        if boxes is not None:
            p.boxes[:n].copy_(boxes, non_blocking=True)
        if flips is not None:
            p.flip[:n].copy_(flips, non_blocking=True)
        else:
            p.flip.zero_()
        return self._backbone()[:n]

    def step(self, images_u8, labels, boxes=None, flips=None):
        feats = self._features(images_u8, labels, boxes, flips).float()
        labels = labels.to(self.dev, non_blocking=True)
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
