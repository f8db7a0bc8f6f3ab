"""Model wrappers that reproduce the reference's state-dict layouts.

* ``FrozenBackboneClassifier`` — the TorchDistributor/DeepSpeed wrappers
  (`02_cifar_torch_distributor_resnet.py:141-159`, `03_tiny_imagenet_torch_distributor_resnet.py:125-143`):
  a ResNet whose backbone is frozen and whose ``fc`` is ``Sequential(Dropout(0.5), Linear)``;
  keys are prefixed ``resnet.`` and the head is ``resnet.fc.1.{weight,bias}``. The reference
  loads ImageNet weights (``weights=DEFAULT``); with no network here the backbone is
  random-init unless a local torchvision-format state dict is supplied.
* ``ComposerResNet50`` — Composer's ``ResNet50(ComposerModel)`` (`03_composer/01_cifar_composer_resnet.ipynb:332-346`):
  keys prefixed ``model.``; ``forward(batch)`` takes ``(inputs, targets)`` and ``loss`` is CE.
  The reference emits 1000 logits for CIFAR-10 (a quirk); ``num_classes`` is
  configurable and defaults to that behaviour for parity.
* ``resnet18_1ch`` — Ray FashionMNIST ResNet-18 with a 1-channel 7x7 stem
  (`05_ray/01_fashion_mnist_pytorch_ray.ipynb:169-174`).
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .resnet import ResNet, register_model, resnet18, resnet50


class FrozenBackboneClassifier(nn.Module):
    def __init__(self, arch: str = "resnet18", num_classes: int = 10, dropout: float = 0.5,
                 freeze_backbone: bool = True, backbone_state: Optional[dict] = None):
        super().__init__()
        self.num_classes = num_classes
        self.resnet: ResNet = {"resnet18": resnet18, "resnet50": resnet50}[arch](num_classes=1000)
        if backbone_state is not None:
            self.resnet.load_state_dict(backbone_state)
        if freeze_backbone:
            for p in self.resnet.parameters():
                p.requires_grad = False
        in_f = self.resnet.fc.in_features
        self.resnet.fc = nn.Sequential(nn.Dropout(dropout), nn.Linear(in_f, num_classes))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.resnet(x)


class ComposerResNet50(nn.Module):
    """Composer-style model: ``forward(batch)`` and ``loss(outputs, batch)``."""

    def __init__(self, num_classes: int = 1000):
        super().__init__()
        self.num_classes = num_classes
        self.model = resnet50(num_classes=num_classes)

    def forward(self, batch):
        inputs = batch[0] if isinstance(batch, (tuple, list)) else batch
        return self.model(inputs)

    def loss(self, outputs: torch.Tensor, batch, label_smoothing: float = 0.0) -> torch.Tensor:
        _, targets = batch
        return F.cross_entropy(outputs, targets, label_smoothing=label_smoothing)


def resnet18_1ch(num_classes: int = 10) -> ResNet:
    return resnet18(num_classes=num_classes, in_channels=1)


register_model("frozen_resnet18", lambda num_classes=10, **kw: FrozenBackboneClassifier("resnet18", num_classes, **kw))
register_model("frozen_resnet50", lambda num_classes=200, **kw: FrozenBackboneClassifier("resnet50", num_classes, **kw))
register_model("composer_resnet50", lambda num_classes=1000, **kw: ComposerResNet50(num_classes))
register_model("resnet18_1ch", lambda num_classes=10, **kw: resnet18_1ch(num_classes))
