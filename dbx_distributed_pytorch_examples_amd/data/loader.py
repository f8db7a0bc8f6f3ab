"""Host -> device input pipeline for the native engine.

Replaces the reference's ``DataLoader(dataset, batch_size, shuffle=True)`` with ``num_workers=0``
and per-sample PIL transforms in the training process (SURVEY.md §3 hot loop item 2, K20, K21):

1. **batch assembly on the host** into a *pinned* uint8 NHWC staging buffer — by the C++ MDS
   reader (``_C.MDSReader.gather``: memcpy of raw pixels, thread pool, GIL released) for MDS
   shards, or by a thread pool over any map-style dataset yielding fixed-size uint8 HWC images;
2. **one async H2D copy per batch** (uint8: 4x fewer PCIe bytes than the reference's fp32 tensors)
   on a dedicated copy stream, double/triple buffered so the copy of batch k+1 overlaps step k;
3. **augmentation on the GPU** inside the captured step: per-sample crop boxes + flips are sampled
   on the host (tiny) and ``augment_u8`` does RandomResizedCrop / RandomCrop(pad) / flip /
   normalise -> bf16 NHWC4 (the native program's stem input).

Ranks read disjoint sample sets (``ShardSampler`` semantics; MDS: ``StreamingDataset.epoch_indices``).
Sized for 288 GB HBM: ``device_cache=True`` keeps a whole uint8 dataset resident on the GPU
(ImageNet-1K at 224x224 is ~193 GB raw, CIFAR/TinyImageNet are trivial) and skips PCIe entirely.
"""
from __future__ import annotations

import math
import random
import threading
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass
from typing import Iterator, Optional, Sequence, Tuple

import numpy as np
import torch

from .transforms import random_resized_crop_box


@dataclass
class AugmentSpec:
    """What the GPU augmentation does per sample (train) — eval uses full-image / center boxes."""
    mode: str = "none"              # none | random_resized_crop | random_crop | center_crop
    scale: Tuple[float, float] = (0.08, 1.0)
    ratio: Tuple[float, float] = (3 / 4, 4 / 3)
    pad: int = 0                    # random_crop padding (CIFAR: 4)
    crop_frac: float = 0.875        # center_crop: 224/256
    hflip: bool = False


def sample_boxes(n: int, hin: int, win: int, hout: int, wout: int, spec: AugmentSpec, rng: random.Random
                 ) -> Tuple[np.ndarray, np.ndarray]:
    """Per-sample crop boxes (top, left, height, width) + horizontal flips for ``augment_u8``,
    vectorised with numpy (a per-sample Python loop costs ~2-4 ms per 512-batch: a loader bottleneck
    at TinyImageNet rates). ``rng`` seeds the batch's numpy generator (reproducible per loader)."""
    g = np.random.default_rng(rng.getrandbits(63))
    boxes = np.zeros((n, 4), np.float32)
    if spec.mode == "random_resized_crop":
        # torchvision's rule: up to 10 tries of (scale, log-ratio), first fitting box wins, else centre
        area = hin * win
        tries = 10
        target = area * g.uniform(spec.scale[0], spec.scale[1], (n, tries))
        ar = np.exp(g.uniform(math.log(spec.ratio[0]), math.log(spec.ratio[1]), (n, tries)))
        cw = np.rint(np.sqrt(target * ar)).astype(np.int64)
        ch = np.rint(np.sqrt(target / ar)).astype(np.int64)
        ok = (cw > 0) & (cw <= win) & (ch > 0) & (ch <= hin)
        first = np.where(ok.any(1), ok.argmax(1), -1)
        rows = np.arange(n)
        h = np.where(first >= 0, ch[rows, np.maximum(first, 0)], 0)
        w = np.where(first >= 0, cw[rows, np.maximum(first, 0)], 0)
        top = (g.random(n) * (hin - h + 1)).astype(np.int64)
        left = (g.random(n) * (win - w + 1)).astype(np.int64)
        # fallback (no try fit): centre crop clamped to the ratio range
        in_ratio = win / hin
        if in_ratio < spec.ratio[0]:
            fw, fh = win, int(round(win / spec.ratio[0]))
        elif in_ratio > spec.ratio[1]:
            fh, fw = hin, int(round(hin * spec.ratio[1]))
        else:
            fw, fh = win, hin
        miss = first < 0
        h[miss], w[miss] = fh, fw
        top[miss], left[miss] = (hin - fh) // 2, (win - fw) // 2
        boxes[:] = np.stack([top, left, h, w], 1)
    elif spec.mode == "random_crop":
        # crop hout x wout from the image zero-padded by `pad` (pad pixels clamp to the edge here)
        boxes[:, 0] = g.integers(-spec.pad, hin + spec.pad - hout + 1, n)
        boxes[:, 1] = g.integers(-spec.pad, win + spec.pad - wout + 1, n)
        boxes[:, 2], boxes[:, 3] = hout, wout
    elif spec.mode == "center_crop":
        h, w = int(round(hin * spec.crop_frac)), int(round(win * spec.crop_frac))
        boxes[:] = ((hin - h) // 2, (win - w) // 2, h, w)
    else:
        boxes[:] = (0, 0, hin, win)
    flips = (g.random(n) < 0.5).astype(np.uint8) if spec.hflip else np.zeros(n, np.uint8)
    return boxes, flips


class NativeImageLoader:
    """Iterates (img_u8 [B,H,W,C] device, labels [B] int64 device, boxes [B,4], flips [B]) per step."""

    def __init__(self, source, batch_size: int, image_hw: Tuple[int, int], device: torch.device,
                 channels: int = 3, indices_fn=None, augment: Optional[AugmentSpec] = None,
                 out_hw: Optional[Tuple[int, int]] = None, drop_last: bool = True, nthreads: int = 8,
                 prefetch: int = 2, seed: int = 0, device_cache: bool = False):
        self.src = source
        self.B = batch_size
        self.H, self.W = image_hw
        self.C = channels
        self.out_hw = out_hw or image_hw
        self.dev = device
        self.aug = augment or AugmentSpec()
        self.drop_last = drop_last
        self.nthreads = nthreads
        self.prefetch = max(1, prefetch)
        self.rng = random.Random(seed)
        self.indices_fn = indices_fn
        self.epoch = 0
        self.native = None
        if hasattr(source, "native_reader"):
            try:
                self.native = source.native_reader()
            except Exception:
                self.native = None  # no extension (CPU host): python gather
        pin = device.type == "cuda"
        self.host = [torch.empty(self.B, self.H, self.W, self.C, dtype=torch.uint8, pin_memory=pin)
                     for _ in range(self.prefetch + 1)]
        self.host_lab = [torch.empty(self.B, dtype=torch.int64, pin_memory=pin) for _ in range(self.prefetch + 1)]
        self.copy_stream = torch.cuda.Stream(device=device) if device.type == "cuda" else None
        self.pool = ThreadPoolExecutor(max_workers=nthreads) if self.native is None else None
        self.cache = None
        if device_cache:
            self._build_device_cache()

    # ------------------------------------------------------------------------------------
    def set_epoch(self, epoch: int):
        self.epoch = epoch
        if hasattr(self.src, "set_epoch"):
            self.src.set_epoch(epoch)

    def _epoch_indices(self) -> np.ndarray:
        if self.indices_fn is not None:
            return np.asarray(self.indices_fn(self.epoch), dtype=np.int64)
        if hasattr(self.src, "epoch_indices"):
            return np.asarray(self.src.epoch_indices(), dtype=np.int64)
        return np.arange(len(self.src), dtype=np.int64)

    def __len__(self) -> int:
        n = len(self._epoch_indices())
        return n // self.B if self.drop_last else math.ceil(n / self.B)

    def _item(self, i: int):
        it = self.src[int(i)]
        if isinstance(it, dict):
            img, y = it["image"], it["label"]
        else:
            img, y = it
        a = np.asarray(img, dtype=np.uint8)
        if a.ndim == 2:
            a = a[:, :, None]
        if a.shape != (self.H, self.W, self.C):
            raise ValueError(f"sample {i}: shape {a.shape}, loader expects {(self.H, self.W, self.C)} "
                             "(resize on the writer side or use a Resize transform)")
        return a, int(y)

    def _fill(self, slot: int, ids: np.ndarray):
        buf, lab = self.host[slot], self.host_lab[slot]
        if self.native is not None:
            self.native.gather(np.ascontiguousarray(ids), buf.data_ptr(), lab.data_ptr(), self.H, self.W, self.C,
                               "image", "label", self.nthreads)
            return
        nb = buf.numpy()
        lb = lab.numpy()

        def one(k):
            a, y = self._item(ids[k])
            nb[k] = a
            lb[k] = y
        list(self.pool.map(one, range(len(ids))))

    def _build_device_cache(self):
        ids = np.arange(len(self.src) if not hasattr(self.src, "num_samples") else self.src.num_samples)
        imgs = torch.empty(len(ids), self.H, self.W, self.C, dtype=torch.uint8, device=self.dev)
        labs = torch.empty(len(ids), dtype=torch.int64, device=self.dev)
        for s in range(0, len(ids), self.B):
            chunk = ids[s:s + self.B]
            self._fill(0, chunk)
            imgs[s:s + len(chunk)].copy_(self.host[0][:len(chunk)])
            labs[s:s + len(chunk)].copy_(self.host_lab[0][:len(chunk)])
        self.cache = (imgs, labs)

    def __iter__(self) -> Iterator:
        ids = self._epoch_indices()
        nb = len(ids) // self.B if self.drop_last else math.ceil(len(ids) / self.B)
        Ho, Wo = self.out_hw
        if self.cache is not None:
            imgs, labs = self.cache
            for b in range(nb):
                sel = torch.from_numpy(ids[b * self.B:(b + 1) * self.B]).to(self.dev)
                boxes, flips = sample_boxes(len(sel), self.H, self.W, Ho, Wo, self.aug, self.rng)
                yield (imgs.index_select(0, sel), labs.index_select(0, sel),
                       torch.from_numpy(boxes).to(self.dev), torch.from_numpy(flips).to(self.dev))
            return
        # host assembly runs ahead in a background thread (bounded by the staging ring)
        ring = len(self.host)
        ready = [threading.Event() for _ in range(nb)]
        errs = []

        def producer():
            try:
                for b in range(nb):
                    if b >= ring:
                        consumed[b - ring].wait()
                    self._fill(b % ring, ids[b * self.B:(b + 1) * self.B])
                    ready[b].set()
            except BaseException as e:  # noqa: BLE001
                errs.append(e)
                for ev in ready:
                    ev.set()

        consumed = [threading.Event() for _ in range(nb)]
        th = threading.Thread(target=producer, daemon=True)
        th.start()
        try:
            for b in range(nb):
                ready[b].wait()
                if errs:
                    raise errs[0]
                slot = b % ring
                n = min(self.B, len(ids) - b * self.B)
                boxes, flips = sample_boxes(n, self.H, self.W, Ho, Wo, self.aug, self.rng)
                if self.copy_stream is not None:
                    with torch.cuda.stream(self.copy_stream):
                        img = self.host[slot][:n].to(self.dev, non_blocking=True)
                        lab = self.host_lab[slot][:n].to(self.dev, non_blocking=True)
                        bx = torch.from_numpy(boxes).to(self.dev, non_blocking=True)
                        fl = torch.from_numpy(flips).to(self.dev, non_blocking=True)
                        ev = torch.cuda.Event()
                        ev.record(self.copy_stream)
                    torch.cuda.current_stream(self.dev).wait_event(ev)
                    for t in (img, lab, bx, fl):
                        t.record_stream(torch.cuda.current_stream(self.dev))
                    # the pinned slot may be refilled once this copy has executed
                    ev.synchronize() if b + ring >= nb else None
                    consumed[b].set() if b + ring >= nb else _set_after(ev, consumed[b])
                else:
                    img = self.host[slot][:n].clone()
                    lab = self.host_lab[slot][:n].clone()
                    bx, fl = torch.from_numpy(boxes), torch.from_numpy(flips)
                    consumed[b].set()
                yield img, lab, bx, fl
        finally:
            for ev in consumed:
                ev.set()
            th.join(timeout=30)


def _set_after(cuda_event, flag: threading.Event):
    """Set ``flag`` once ``cuda_event`` completes, without blocking the training thread."""
    def waiter():
        cuda_event.synchronize()
        flag.set()
    threading.Thread(target=waiter, daemon=True).start()
