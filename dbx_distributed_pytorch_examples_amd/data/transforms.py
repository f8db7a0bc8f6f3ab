"""Image transforms (torchvision is not installed on this image).

CPU-side, torchvision-compatible semantics for the transforms the reference uses
(`utils/hf_dataset_utilities.py:58-81`, `03_composer/01_cifar_composer_resnet.ipynb:207-215`,
`02_deepspeed/03_1k_imagenet_deepspeed_resnet.py:43-53`): Compose, Resize, CenterCrop,
RandomCrop(pad), RandomResizedCrop, RandomHorizontalFlip, Grayscale, ToTensor, Normalize, Lambda.
Inputs: PIL images or uint8 HWC numpy arrays.

For the native engine the heavy per-sample work moves to the GPU instead: the loader ships
uint8 HWC batches and ``ops.kernels.augment_u8`` does crop / bilinear resize / flip /
normalise into bf16 NHWC4 — the CPU only decodes.

Quirk NOT replicated: the reference applies train-time random augmentation
to validation data (``default_image_transforms`` for the test split); ``default_image_transforms
(train=False)`` here is deterministic.
"""
from __future__ import annotations

import math
import random
from typing import Callable, List, Sequence, Tuple, Union

import numpy as np
import torch

try:
    from PIL import Image
except Exception:  # pragma: no cover
    Image = None

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)
CIFAR_MEAN = (0.4914, 0.4822, 0.4465)
CIFAR_STD = (0.2470, 0.2435, 0.2616)
MNIST_MEAN, MNIST_STD = (0.1307,), (0.3081,)


def _to_pil(img):
    if Image is not None and isinstance(img, Image.Image):
        return img
    a = np.asarray(img)
    if a.ndim == 3 and a.shape[2] == 1:
        a = a[..., 0]
    return Image.fromarray(a)


def _size(img) -> Tuple[int, int]:  # (w, h)
    if Image is not None and isinstance(img, Image.Image):
        return img.size
    a = np.asarray(img)
    return a.shape[1], a.shape[0]


class Compose:
    def __init__(self, transforms: Sequence[Callable]):
        self.transforms = list(transforms)

    def __call__(self, x):
        for t in self.transforms:
            x = t(x)
        return x


class Lambda:
    def __init__(self, fn):
        self.fn = fn

    def __call__(self, x):
        return self.fn(x)


class Resize:
    """``Resize((h, w))`` exact, or ``Resize(s)`` = shorter side to s (bilinear)."""

    def __init__(self, size):
        self.size = size

    def __call__(self, img):
        img = _to_pil(img)
        w, h = img.size
        if isinstance(self.size, int):
            if w <= h:
                nw, nh = self.size, int(round(h * self.size / w))
            else:
                nh, nw = self.size, int(round(w * self.size / h))
        else:
            nh, nw = self.size
        return img.resize((nw, nh), Image.BILINEAR)


class CenterCrop:
    def __init__(self, size):
        self.size = (size, size) if isinstance(size, int) else tuple(size)

    def __call__(self, img):
        img = _to_pil(img)
        w, h = img.size
        th, tw = self.size
        left, top = int(round((w - tw) / 2.0)), int(round((h - th) / 2.0))
        return img.crop((left, top, left + tw, top + th))


class RandomCrop:
    def __init__(self, size, padding: int = 0):
        self.size = (size, size) if isinstance(size, int) else tuple(size)
        self.padding = padding

    def __call__(self, img):
        a = np.asarray(_to_pil(img))
        if self.padding:
            pad = [(self.padding, self.padding), (self.padding, self.padding)] + ([(0, 0)] if a.ndim == 3 else [])
            a = np.pad(a, pad)
        h, w = a.shape[:2]
        th, tw = self.size
        i, j = random.randint(0, h - th), random.randint(0, w - tw)
        return Image.fromarray(np.ascontiguousarray(a[i:i + th, j:j + tw]))


def random_resized_crop_box(w: int, h: int, scale=(0.08, 1.0), ratio=(3 / 4, 4 / 3), rng=random):
    """torchvision's RandomResizedCrop box sampling: returns (top, left, height, width)."""
    area = h * w
    log_r = (math.log(ratio[0]), math.log(ratio[1]))
    for _ in range(10):
        target = area * rng.uniform(*scale)
        ar = math.exp(rng.uniform(*log_r))
        cw = int(round(math.sqrt(target * ar)))
        ch = int(round(math.sqrt(target / ar)))
        if 0 < cw <= w and 0 < ch <= h:
            return rng.randint(0, h - ch), rng.randint(0, w - cw), ch, cw
    in_ratio = w / h
    if in_ratio < ratio[0]:
        cw, ch = w, int(round(w / ratio[0]))
    elif in_ratio > ratio[1]:
        ch, cw = h, int(round(h * ratio[1]))
    else:
        cw, ch = w, h
    return (h - ch) // 2, (w - cw) // 2, ch, cw


class RandomResizedCrop:
    def __init__(self, size, scale=(0.08, 1.0), ratio=(3 / 4, 4 / 3)):
        self.size = (size, size) if isinstance(size, int) else tuple(size)
        self.scale, self.ratio = scale, ratio

    def __call__(self, img):
        img = _to_pil(img)
        w, h = img.size
        t, l, ch, cw = random_resized_crop_box(w, h, self.scale, self.ratio)
        return img.resize(self.size[::-1], Image.BILINEAR, box=(l, t, l + cw, t + ch))


class RandomHorizontalFlip:
    def __init__(self, p: float = 0.5):
        self.p = p

    def __call__(self, img):
        if random.random() < self.p:
            img = _to_pil(img)
            return img.transpose(Image.FLIP_LEFT_RIGHT)
        return img


class Grayscale:
    def __init__(self, num_output_channels: int = 1):
        self.n = num_output_channels

    def __call__(self, img):
        g = _to_pil(img).convert("L")
        return g.convert("RGB") if self.n == 3 else g


class ToTensor:
    """PIL / uint8 HWC -> float CHW in [0, 1]."""

    def __call__(self, img):
        a = np.asarray(_to_pil(img) if not isinstance(img, np.ndarray) else img)
        if a.ndim == 2:
            a = a[:, :, None]
        return torch.from_numpy(np.array(a.transpose(2, 0, 1), copy=True)).float().div_(255.0)


class PILToUint8HWC:
    """Decode only: PIL -> uint8 HWC numpy (the native loader's CPU transform)."""

    def __init__(self, channels: int = 3):
        self.channels = channels

    def __call__(self, img):
        img = _to_pil(img)
        img = img.convert("RGB" if self.channels == 3 else "L")
        a = np.asarray(img)
        return a if a.ndim == 3 else a[:, :, None]


class Normalize:
    def __init__(self, mean, std):
        self.mean = torch.tensor(mean).view(-1, 1, 1)
        self.std = torch.tensor(std).view(-1, 1, 1)

    def __call__(self, t: torch.Tensor):
        return (t - self.mean) / self.std


def gray_to_rgb(x: torch.Tensor) -> torch.Tensor:
    return x.repeat(3, 1, 1) if x.size(0) == 1 else x


def default_image_transforms(image_size: int, normalize_transform: bool = True, convert_rgb: bool = True,
                             train: bool = True, grayscale_first: bool = False) -> Compose:
    """`utils/hf_dataset_utilities.py:58-81` (+ the 03a variant's leading ``Grayscale(3)``, `03a…:116`)."""
    t: List[Callable] = []
    if grayscale_first:
        t.append(Grayscale(3))
    t.append(Resize((image_size, image_size)))
    if train:
        t.append(RandomHorizontalFlip())
    t.append(ToTensor())
    if convert_rgb:
        t.append(Lambda(gray_to_rgb))
    if normalize_transform:
        t.append(Normalize(IMAGENET_MEAN, IMAGENET_STD))
    return Compose(t)


def cifar_transforms(train: bool = True) -> Compose:
    if train:
        return Compose([RandomCrop(32, padding=4), RandomHorizontalFlip(), ToTensor(), Normalize(CIFAR_MEAN, CIFAR_STD)])
    return Compose([ToTensor(), Normalize(CIFAR_MEAN, CIFAR_STD)])


def imagenet_transforms(train: bool = True, size: int = 224) -> Compose:
    if train:
        return Compose([RandomResizedCrop(size), RandomHorizontalFlip(), ToTensor(), Normalize(IMAGENET_MEAN, IMAGENET_STD)])
    return Compose([Resize(int(size * 256 / 224)), CenterCrop(size), ToTensor(), Normalize(IMAGENET_MEAN, IMAGENET_STD)])


def mnist_transforms(fashion: bool = False) -> Compose:
    m, s = ((0.5,), (0.5,)) if fashion else (MNIST_MEAN, MNIST_STD)
    return Compose([ToTensor(), Normalize(m, s)])
