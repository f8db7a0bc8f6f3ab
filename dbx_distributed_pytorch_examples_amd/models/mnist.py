"""LeNet-style MNIST ``Net`` (`/root/reference/01_torch_distributor/01_basic_torch_distributor.py:75-91`).

conv5x5(1->10) -> maxpool2 -> ReLU -> conv5x5(10->20) -> Dropout2d -> maxpool2 -> ReLU
-> fc 320->50 -> ReLU -> dropout -> fc 50->10 -> log_softmax. 21,840 parameters; keys
``conv1, conv2, fc1, fc2`` so the reference's ``checkpoint-{epoch}.pth.tar`` files load.
The reference calls ``F.log_softmax(x)`` without ``dim`` (implicit dim=1 for 2-D); we pass
``dim=1`` explicitly (same result, no deprecation warning).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .resnet import register_model


class Net(nn.Module):
    def __init__(self, num_classes: int = 10):
        super().__init__()
        self.num_classes = num_classes
        self.conv1 = nn.Conv2d(1, 10, kernel_size=5)
        self.conv2 = nn.Conv2d(10, 20, kernel_size=5)
        self.conv2_drop = nn.Dropout2d()
        self.fc1 = nn.Linear(320, 50)
        self.fc2 = nn.Linear(50, num_classes)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = F.relu(F.max_pool2d(self.conv1(x), 2))
        x = F.relu(F.max_pool2d(self.conv2_drop(self.conv2(x)), 2))
        x = x.view(-1, 320)
        x = F.relu(self.fc1(x))
        x = F.dropout(x, training=self.training)
        x = self.fc2(x)
        return F.log_softmax(x, dim=1)


register_model("mnist_net", lambda num_classes=10, **kw: Net(num_classes))
