"""ResNet family with torchvision-compatible parameter names.

The reference pulls its ResNets from torchvision (`models.resnet18/50`, e.g.
`/root/reference/01_torch_distributor/02_cifar_torch_distributor_resnet.py:141-159`,
`/root/reference/04_accelerate/01_cifar_accelerate.ipynb:475-479`,
`/root/reference/05_ray/02_cifar_resnet_pytorch_ray.ipynb:278-280`) and defines a
CIFAR-stem ResNet-18 in `/root/reference/setup/resnet18.py:3-67`. torchvision is not
available on this image, so the architectures are written here directly. State-dict
keys and parameter counts match torchvision exactly (tests/test_models.py pins
11,181,642 / 23,528,522 / 25,557,032 params), so checkpoints move both ways.

Layout: these are ordinary ``nn.Module`` s (NCHW API, any device). On a GPU the
training engine (``dbx.engine``) re-plans them as NHWC bf16 programs that run the
hand-written HIP kernels in ``dbx.ops``; on CPU they run stock PyTorch ops. The
module tree is therefore the single source of truth for parameters/state dicts.
"""
from __future__ import annotations

import math
from typing import Callable, List, Optional, Sequence, Type, Union

import torch
import torch.nn as nn
import torch.nn.functional as F

__all__ = [
    "BasicBlock", "Bottleneck", "ResNet", "resnet18", "resnet34", "resnet50",
    "resnet101", "resnet152", "CifarBlock", "CifarResNet18", "build_model",
]


def conv3x3(cin: int, cout: int, stride: int = 1) -> nn.Conv2d:
    return nn.Conv2d(cin, cout, kernel_size=3, stride=stride, padding=1, bias=False)


def conv1x1(cin: int, cout: int, stride: int = 1) -> nn.Conv2d:
    return nn.Conv2d(cin, cout, kernel_size=1, stride=stride, bias=False)


class BasicBlock(nn.Module):
    """torchvision BasicBlock (two 3x3 convs), keys conv1/bn1/conv2/bn2/downsample.{0,1}."""

    expansion = 1

    def __init__(self, inplanes: int, planes: int, stride: int = 1,
                 downsample: Optional[nn.Module] = None):
        super().__init__()
        self.conv1 = conv3x3(inplanes, planes, stride)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = conv3x3(planes, planes)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        identity = x
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        if self.downsample is not None:
            identity = self.downsample(x)
        return self.relu(out + identity)


class Bottleneck(nn.Module):
    """torchvision v1.5 Bottleneck: stride lives on the 3x3 conv (SURVEY.md §2.4 note)."""

    expansion = 4

    def __init__(self, inplanes: int, planes: int, stride: int = 1,
                 downsample: Optional[nn.Module] = None):
        super().__init__()
        width = planes
        self.conv1 = conv1x1(inplanes, width)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = conv3x3(width, width, stride)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = conv1x1(width, planes * self.expansion)
        self.bn3 = nn.BatchNorm2d(planes * self.expansion)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        identity = x
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        if self.downsample is not None:
            identity = self.downsample(x)
        return self.relu(out + identity)


class ResNet(nn.Module):
    """torchvision-compatible ResNet.

    ``in_channels`` != 3 reproduces the Ray FashionMNIST variant that swaps conv1 for
    ``Conv2d(1, 64, 7, 2, 3)`` (`/root/reference/05_ray/01_fashion_mnist_pytorch_ray.ipynb:169-174`).
    """

    def __init__(self, block: Type[Union[BasicBlock, Bottleneck]], layers: Sequence[int],
                 num_classes: int = 1000, in_channels: int = 3,
                 zero_init_residual: bool = False):
        super().__init__()
        self.block_type = block
        self.layers_cfg = list(layers)
        self.num_classes = num_classes
        self.inplanes = 64
        self.conv1 = nn.Conv2d(in_channels, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        init_resnet_(self, zero_init_residual)

    def _make_layer(self, block, planes: int, blocks: int, stride: int = 1) -> nn.Sequential:
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(
                conv1x1(self.inplanes, planes * block.expansion, stride),
                nn.BatchNorm2d(planes * block.expansion),
            )
        layers: List[nn.Module] = [block(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes))
        return nn.Sequential(*layers)

    def forward_features(self, x: torch.Tensor) -> torch.Tensor:
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return torch.flatten(self.avgpool(x), 1)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.fc(self.forward_features(x))


def init_resnet_(model: nn.Module, zero_init_residual: bool = False) -> None:
    """torchvision initialisation: kaiming-normal(fan_out) convs, BN (1, 0), default Linear."""
    for m in model.modules():
        if isinstance(m, nn.Conv2d):
            nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
        elif isinstance(m, (nn.BatchNorm2d, nn.GroupNorm)):
            nn.init.constant_(m.weight, 1)
            nn.init.constant_(m.bias, 0)
    if zero_init_residual:
        for m in model.modules():
            if isinstance(m, Bottleneck):
                nn.init.constant_(m.bn3.weight, 0)
            elif isinstance(m, BasicBlock):
                nn.init.constant_(m.bn2.weight, 0)


def resnet18(num_classes: int = 1000, **kw) -> ResNet:
    return ResNet(BasicBlock, [2, 2, 2, 2], num_classes=num_classes, **kw)


def resnet34(num_classes: int = 1000, **kw) -> ResNet:
    return ResNet(BasicBlock, [3, 4, 6, 3], num_classes=num_classes, **kw)


def resnet50(num_classes: int = 1000, **kw) -> ResNet:
    return ResNet(Bottleneck, [3, 4, 6, 3], num_classes=num_classes, **kw)


def resnet101(num_classes: int = 1000, **kw) -> ResNet:
    return ResNet(Bottleneck, [3, 4, 23, 3], num_classes=num_classes, **kw)


def resnet152(num_classes: int = 1000, **kw) -> ResNet:
    return ResNet(Bottleneck, [3, 8, 36, 3], num_classes=num_classes, **kw)


# --------------------------------------------------------------------------------------
# CIFAR-stem ResNet-18 of /root/reference/setup/resnet18.py (keys: conv1, bn1,
# layer{1-4}.{0,1}.{conv1,bn1,conv2,bn2,skip_connection.{0,1}}, fc — SURVEY.md §5.4).
# --------------------------------------------------------------------------------------
class CifarBlock(nn.Module):
    """Residual block of `setup/resnet18.py:3-27` (skip = 1x1 conv + BN when shape changes)."""

    def __init__(self, cin: int, cout: int, stride: int = 1):
        super().__init__()
        self.conv1 = conv3x3(cin, cout, stride)
        self.bn1 = nn.BatchNorm2d(cout)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = conv3x3(cout, cout)
        self.bn2 = nn.BatchNorm2d(cout)
        self.skip_connection = nn.Sequential()
        if stride != 1 or cin != cout:
            self.skip_connection = nn.Sequential(conv1x1(cin, cout, stride), nn.BatchNorm2d(cout))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        return self.relu(out + self.skip_connection(x))


class CifarResNet18(nn.Module):
    """3x3-s1 stem + maxpool + 4x2 CifarBlocks + avgpool + fc (`setup/resnet18.py:29-67`)."""

    def __init__(self, num_classes: int = 10, in_channels: int = 3):
        super().__init__()
        self.num_classes = num_classes
        self.conv1 = nn.Conv2d(in_channels, 64, kernel_size=3, stride=1, padding=1, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        cin = 64
        for i, (cout, stride) in enumerate([(64, 1), (128, 2), (256, 2), (512, 2)]):
            blocks = [CifarBlock(cin, cout, stride), CifarBlock(cout, cout, 1)]
            setattr(self, f"layer{i + 1}", nn.Sequential(*blocks))
            cin = cout
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512, num_classes)

    def forward_features(self, x: torch.Tensor) -> torch.Tensor:
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return torch.flatten(self.avgpool(x), 1)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.fc(self.forward_features(x))


_FACTORIES: dict = {
    "resnet18": resnet18, "resnet34": resnet34, "resnet50": resnet50,
    "resnet101": resnet101, "resnet152": resnet152,
    "cifar_resnet18": lambda num_classes=10, **kw: CifarResNet18(num_classes, **kw),
}


def build_model(name: str, num_classes: int = 1000, **kw) -> nn.Module:
    """Factory used by configs/CLI: ``build_model("resnet50", 1000)``."""
    from . import mnist, wrappers  # noqa: F401  (register extra names)
    key = name.lower()
    if key not in _FACTORIES:
        raise KeyError(f"unknown model {name!r}; known: {sorted(_FACTORIES)}")
    m = _FACTORIES[key](num_classes=num_classes, **kw)
    # factory spec: lets checkpoint / MLflow loaders rebuild the module without unpickling code
    m._dbx_spec = {"name": key, "kwargs": dict(num_classes=num_classes, **{k: v for k, v in kw.items()
                                                                          if isinstance(v, (int, float, str, bool))})}
    return m


def register_model(name: str, factory: Callable[..., nn.Module]) -> None:
    _FACTORIES[name.lower()] = factory
