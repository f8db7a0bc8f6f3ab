"""Datasets: synthetic, MNIST/FashionMNIST (IDX), CIFAR-10 (binary), image folders.

The reference pulls everything from the HF Hub or torchvision downloads
(`01_basic_torch_distributor.py:278-286`, `05_ray/01_fashion_mnist_pytorch_ray.ipynb:180-185`,
`utils/hf_dataset_utilities.py:8-18`). There is no network here, so every dataset reads local
files in its canonical on-disk format, and :class:`SyntheticImages` stands in for ImageNet-shaped
data in benchmarks (random uint8 images + labels, deterministic per index).

All datasets return ``(image, label)`` where image is whatever the ``transform`` makes of a PIL
image (default: uint8 HWC numpy, the native loader's input format).
"""
from __future__ import annotations

import gzip
import os
import struct
from typing import Callable, List, Optional, Tuple

import numpy as np
import torch
from torch.utils.data import Dataset

try:
    from PIL import Image
except Exception:  # pragma: no cover
    Image = None


class SyntheticImages(Dataset):
    """Deterministic random uint8 HWC images + labels (ImageNet / CIFAR shaped)."""

    def __init__(self, n: int, image_size: int = 224, channels: int = 3, num_classes: int = 1000,
                 seed: int = 0, transform: Optional[Callable] = None):
        self.n, self.size, self.c, self.num_classes, self.seed = n, image_size, channels, num_classes, seed
        self.transform = transform
        g = np.random.default_rng(seed)
        self.labels = g.integers(0, num_classes, size=n).astype(np.int64)

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        g = np.random.default_rng(self.seed * 1_000_003 + i)
        img = g.integers(0, 256, size=(self.size, self.size, self.c), dtype=np.uint8)
        if self.transform is not None:
            img = self.transform(Image.fromarray(img if self.c == 3 else img[..., 0]))
        return img, int(self.labels[i])


def learnable_synthetic(n: int, image_size: int, num_classes: int, seed: int = 0, noise: float = 48.0,
                        device=None, proto_res: int = 8):
    """A learnable synthetic classification task (for accuracy checks without a dataset): every
    class has a fixed random low-resolution RGB prototype (``proto_res``^2, bilinearly upsampled);
    a sample is its class prototype under a random brightness/contrast change, a random shift of
    up to 1/8 of the image and Gaussian pixel noise (std ``noise`` in 0..255 units). Returns uint8
    NHWC images [n, S, S, 3] and int64 labels, generated on ``device`` (deterministic in seed)."""
    import torch
    import torch.nn.functional as F
    g = torch.Generator(device="cpu").manual_seed(seed)
    protos = torch.rand(num_classes, 3, proto_res, proto_res, generator=torch.Generator().manual_seed(12345)) * 255
    protos = F.interpolate(protos, size=(image_size, image_size), mode="bilinear", align_corners=False)
    labels = torch.randint(0, num_classes, (n,), generator=g)
    gain = 0.7 + 0.6 * torch.rand(n, 1, 1, 1, generator=g)
    bias = (torch.rand(n, 1, 1, 1, generator=g) - 0.5) * 60
    sh = image_size // 8
    dy = torch.randint(-sh, sh + 1, (n,), generator=g)
    dx = torch.randint(-sh, sh + 1, (n,), generator=g)
    out = torch.empty(n, image_size, image_size, 3, dtype=torch.uint8)
    for i0 in range(0, n, 1024):
        sl = slice(i0, min(n, i0 + 1024))
        x = protos[labels[sl]] * gain[sl] + bias[sl]
        x = torch.stack([torch.roll(xi, shifts=(int(a), int(b)), dims=(1, 2)) for xi, a, b in zip(x, dy[sl], dx[sl])])
        x = x + noise * torch.randn(x.shape, generator=g)
        out[sl] = x.clamp_(0, 255).round_().to(torch.uint8).permute(0, 2, 3, 1)
    if device is not None:
        out, labels = out.to(device), labels.to(device)
    return out, labels


def _open(path):
    return gzip.open(path, "rb") if path.endswith(".gz") else open(path, "rb")


def read_idx(path: str) -> np.ndarray:
    """IDX file (MNIST format): magic (0,0,dtype,ndim), dims big-endian uint32, data."""
    with _open(path) as f:
        data = f.read()
    zero, dtype, ndim = struct.unpack(">HBB", data[:4])
    if zero != 0 or dtype != 0x08:
        raise ValueError(f"{path}: not a uint8 IDX file")
    dims = struct.unpack(">" + "I" * ndim, data[4:4 + 4 * ndim])
    return np.frombuffer(data, dtype=np.uint8, offset=4 + 4 * ndim).reshape(dims)


def write_idx(path: str, arr: np.ndarray) -> None:
    arr = np.ascontiguousarray(arr, dtype=np.uint8)
    with open(path, "wb") as f:
        f.write(struct.pack(">HBB", 0, 0x08, arr.ndim))
        f.write(struct.pack(">" + "I" * arr.ndim, *arr.shape))
        f.write(arr.tobytes())


class MNIST(Dataset):
    """MNIST / FashionMNIST from the standard IDX files under ``root`` (raw/ or flat, .gz ok)."""

    files = {True: ("train-images-idx3-ubyte", "train-labels-idx1-ubyte"),
             False: ("t10k-images-idx3-ubyte", "t10k-labels-idx1-ubyte")}

    def __init__(self, root: str, train: bool = True, transform: Optional[Callable] = None, **_):
        img_f, lab_f = self.files[train]
        self.images = read_idx(self._find(root, img_f))
        self.labels = read_idx(self._find(root, lab_f)).astype(np.int64)
        self.transform = transform
        self.num_classes = 10

    @staticmethod
    def _find(root, name):
        for sub in ("", "raw", "MNIST/raw", "FashionMNIST/raw"):
            for ext in ("", ".gz"):
                p = os.path.join(root, sub, name + ext)
                if os.path.exists(p):
                    return p
        raise FileNotFoundError(f"{name} not found under {root}")

    def __len__(self):
        return len(self.labels)

    def __getitem__(self, i):
        img = self.images[i]
        if self.transform is not None:
            img = self.transform(Image.fromarray(img))
        else:
            img = img[:, :, None]
        return img, int(self.labels[i])


FashionMNIST = MNIST


class CIFAR10(Dataset):
    """CIFAR-10 binary version (``data_batch_{1..5}.bin`` / ``test_batch.bin``: 1 label byte +
    3072 CHW pixel bytes per record). No pickle files are read."""

    def __init__(self, root: str, train: bool = True, transform: Optional[Callable] = None, **_):
        names = [f"data_batch_{i}.bin" for i in range(1, 6)] if train else ["test_batch.bin"]
        base = root
        for sub in ("", "cifar-10-batches-bin"):
            if os.path.exists(os.path.join(root, sub, names[0])):
                base = os.path.join(root, sub)
        recs = [np.fromfile(os.path.join(base, n), dtype=np.uint8).reshape(-1, 3073) for n in names]
        r = np.concatenate(recs)
        self.labels = r[:, 0].astype(np.int64)
        self.images = r[:, 1:].reshape(-1, 3, 32, 32).transpose(0, 2, 3, 1).copy()  # HWC
        self.transform = transform
        self.num_classes = 10

    def __len__(self):
        return len(self.labels)

    def __getitem__(self, i):
        img = self.images[i]
        if self.transform is not None:
            img = self.transform(Image.fromarray(img))
        return img, int(self.labels[i])


def write_cifar10_bin(path: str, images_hwc: np.ndarray, labels: np.ndarray) -> None:
    recs = np.concatenate([labels.astype(np.uint8)[:, None],
                           images_hwc.transpose(0, 3, 1, 2).reshape(len(labels), -1)], axis=1)
    recs.astype(np.uint8).tofile(path)


IMG_EXT = (".jpg", ".jpeg", ".png", ".bmp", ".webp", ".JPEG")


class ImageFolder(Dataset):
    """``root/<class>/<img>`` layout (ImageNet train, TinyImageNet train/<wnid>/images/)."""

    def __init__(self, root: str, transform: Optional[Callable] = None, **_):
        self.classes = sorted(d for d in os.listdir(root) if os.path.isdir(os.path.join(root, d)))
        self.class_to_idx = {c: i for i, c in enumerate(self.classes)}
        self.samples: List[Tuple[str, int]] = []
        for c in self.classes:
            for dp, _, fns in os.walk(os.path.join(root, c)):
                for fn in sorted(fns):
                    if fn.endswith(IMG_EXT):
                        self.samples.append((os.path.join(dp, fn), self.class_to_idx[c]))
        self.transform = transform
        self.num_classes = len(self.classes)

    def __len__(self):
        return len(self.samples)

    def __getitem__(self, i):
        p, y = self.samples[i]
        img = Image.open(p).convert("RGB")
        if self.transform is not None:
            img = self.transform(img)
        return img, y


def build_dataset(name: str, root: str = "", train: bool = True, transform=None, image_size: int = 224,
                  num_classes: int = 1000, n_synthetic: int = 0, seed: int = 0) -> Dataset:
    name = name.lower()
    if name == "synthetic":
        return SyntheticImages(n_synthetic or 1024, image_size, 3, num_classes, seed=seed + (0 if train else 1),
                               transform=transform)
    if name in ("mnist", "fashion_mnist", "fashionmnist"):
        return MNIST(root, train, transform)
    if name in ("cifar10", "cifar"):
        return CIFAR10(root, train, transform)
    if name in ("folder", "imagenet", "tiny_imagenet"):
        return ImageFolder(os.path.join(root, "train" if train else "val"), transform)
    raise KeyError(f"unknown dataset {name!r}")


# ----------------------------------------------------------------------------------------
# Dataset snapshots (`03a…:157-158` pickles whole Dataset objects with torch.save,
# which only loads with weights_only=False). Here a snapshot is plain tensors — uint8 HWC images
# and int64 labels — loadable with torch.load(weights_only=True).
def save_tensor_dataset(ds, path: str, max_items: Optional[int] = None) -> str:
    n = len(ds) if max_items is None else min(len(ds), max_items)
    imgs, labels = [], []
    for i in range(n):
        img, y = ds[i]
        if isinstance(img, torch.Tensor):
            t = img
            if t.is_floating_point():
                t = (t.clamp(0, 1) * 255).round().to(torch.uint8)
            if t.dim() == 3 and t.shape[0] in (1, 3) and t.shape[-1] not in (1, 3):
                t = t.permute(1, 2, 0)
        else:
            arr = np.asarray(img)
            t = torch.from_numpy(np.ascontiguousarray(arr if arr.ndim == 3 else arr[:, :, None]))
        imgs.append(t.contiguous())
        labels.append(int(y))
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    torch.save({"images": torch.stack(imgs), "labels": torch.tensor(labels, dtype=torch.int64)}, path)
    return path


class TensorImageDataset(Dataset):
    """A ``save_tensor_dataset`` snapshot (uint8 HWC) with an optional transform."""

    def __init__(self, path: str, transform=None):
        d = torch.load(path, weights_only=True)
        self.images, self.labels, self.transform = d["images"], d["labels"], transform
        self.num_classes = int(self.labels.max().item()) + 1 if len(self.labels) else 0

    def __len__(self) -> int:
        return len(self.labels)

    def __getitem__(self, i):
        img = self.images[i]
        if self.transform is not None:
            img = self.transform(img.numpy())
        return img, int(self.labels[i])
