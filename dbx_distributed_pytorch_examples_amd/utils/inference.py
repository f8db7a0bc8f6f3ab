"""Inference sanity check and GPU memory release.

The reference ends each example with a single-image prediction (`02_cifar…:366-387`,
``predict_image`` in `03a…:660-707`): ``ToTensor()(image)`` → ``model(x.unsqueeze(0))`` →
``torch.max`` and a print of predicted vs true. It applies **no Normalize** although training
normalised (a train/test mismatch); ``predict_image`` normalises by default and
keeps ``normalize=False`` to reproduce the reference's behaviour. ``release_gpu_memory`` replaces
``dbutils.library.restartPython()`` (`01_basic…:387`): drop cached blocks, collect, and report.
"""
from __future__ import annotations

import gc
from typing import Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn as nn

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def image_to_tensor(image, size: Optional[int] = None, normalize: bool = True,
                    mean: Sequence[float] = IMAGENET_MEAN, std: Sequence[float] = IMAGENET_STD) -> torch.Tensor:
    """PIL image / HWC uint8 array / CHW float tensor -> [1, C, H, W] float32."""
    if isinstance(image, torch.Tensor):
        x = image.float()
        if x.dim() == 3 and x.shape[-1] in (1, 3) and x.shape[0] not in (1, 3):
            x = x.permute(2, 0, 1)
        if x.max() > 1.5:
            x = x / 255.0
    else:
        arr = np.asarray(image.convert("RGB") if hasattr(image, "convert") else image)
        if arr.ndim == 2:
            arr = arr[:, :, None]
        x = torch.from_numpy(np.ascontiguousarray(arr)).permute(2, 0, 1).float() / 255.0
    if x.dim() == 2:
        x = x[None]
    if size is not None and tuple(x.shape[-2:]) != (size, size):
        x = torch.nn.functional.interpolate(x[None], size=(size, size), mode="bilinear", align_corners=False)[0]
    if normalize:
        c = x.shape[0]
        m = torch.tensor(mean[:c] if len(mean) >= c else mean * c).view(-1, 1, 1)
        s = torch.tensor(std[:c] if len(std) >= c else std * c).view(-1, 1, 1)
        x = (x - m) / s
    return x[None]


@torch.no_grad()
def predict_image(model: nn.Module, image, device=None, size: Optional[int] = None, normalize: bool = True,
                  classes: Optional[Sequence[str]] = None, true_label=None, verbose: bool = True
                  ) -> Tuple[int, float]:
    """Predicted class index and its softmax probability for one image."""
    device = device or next(model.parameters()).device
    was_training = model.training
    model.eval()
    x = image_to_tensor(image, size=size, normalize=normalize).to(device)
    logits = model(x).float()
    prob = torch.softmax(logits, dim=1)
    p, idx = torch.max(prob, 1)
    model.train(was_training)
    pred = int(idx.item())
    if verbose:
        name = classes[pred] if classes else pred
        tl = (classes[true_label] if classes and true_label is not None else true_label)
        print(f"Predicted: {name} (p={float(p):.3f})" + (f"  True: {tl}" if true_label is not None else ""))
    return pred, float(p)


def release_gpu_memory(verbose: bool = False) -> dict:
    """Free cached device memory held by this process (the notebook restart of the reference)."""
    gc.collect()
    out = {"allocated": 0, "reserved": 0}
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        out = {"allocated": torch.cuda.memory_allocated(), "reserved": torch.cuda.memory_reserved()}
    if verbose:
        print(f"GPU memory after release: {out}")
    return out
