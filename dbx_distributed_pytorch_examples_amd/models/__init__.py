from .resnet import (BasicBlock, Bottleneck, ResNet, CifarBlock, CifarResNet18, build_model,
                     register_model, resnet18, resnet34, resnet50, resnet101, resnet152)
from .mnist import Net
from .wrappers import ComposerResNet50, FrozenBackboneClassifier, resnet18_1ch

__all__ = [
    "BasicBlock", "Bottleneck", "ResNet", "CifarBlock", "CifarResNet18", "build_model",
    "register_model", "resnet18", "resnet34", "resnet50", "resnet101", "resnet152", "Net",
    "ComposerResNet50", "FrozenBackboneClassifier", "resnet18_1ch",
]
