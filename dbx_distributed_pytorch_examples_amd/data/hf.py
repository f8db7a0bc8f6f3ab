"""Hugging Face dataset utilities — API of `/root/reference/utils/hf_dataset_utilities.py`.

``hfds_download_volume`` (`:8-18`), ``hf_get_num_classes`` (`:20-28`), ``create_torch_image_dataset``
(`:31-55`) and ``default_image_transforms`` (`:58-81`, in data.transforms). There is no network on
this image: ``load_dataset`` works from a local HF cache / local files only (``HF_DATASETS_OFFLINE``
is forced on). ``create_torch_image_dataset`` returns a class the standard pickler handles (registered
on this module by a name derived from the column names and re-created on demand in a fresh process);
the reference's closure class cannot be pickled, which is why `03a…:80-97` re-defines it inline.
"""
from __future__ import annotations

import os
from typing import Any, Optional

from torch.utils.data import Dataset

from .transforms import default_image_transforms  # noqa: F401  (re-export: reference API)


def hfds_download_volume(hf_cache: str, dataset_path: str, trust_remote_code: bool = False,
                         disable_progress: bool = False, **kw):
    os.environ.setdefault("HF_DATASETS_OFFLINE", "1")
    import datasets
    if disable_progress:
        datasets.disable_progress_bars()
    return datasets.load_dataset(path=dataset_path, cache_dir=hf_cache, trust_remote_code=trust_remote_code, **kw)


def hf_get_num_classes(dataset, split_key: str, label_key: str = "label") -> int:
    return len(set(dataset[split_key][label_key]))


class HFImageDataset(Dataset):
    """Torch dataset over an HF split (columns materialised once, like the reference)."""

    def __init__(self, data, transform=None, image_key: str = "image", label_key: str = "label"):
        self.images = data[image_key]
        self.labels = data[label_key]
        self.transform = transform
        self.num_classes = len(set(self.labels))

    def __len__(self) -> int:
        return len(self.images)

    def __getitem__(self, idx):
        image = self.images[idx]
        if self.transform:
            image = self.transform(image)
        return image, self.labels[idx]


_CLASSES: dict = {}
_PREFIX = "HFImageDataset__"


def _class_name(image_key: str, label_key: str) -> str:
    # hex of the column names: any names give a valid, dot-free attribute name pickle can resolve
    return f"{_PREFIX}{image_key.encode().hex()}__{label_key.encode().hex()}"


def create_torch_image_dataset(image_key: str, label_key: str):
    """Returns a dataset *class* bound to the column names (reference signature,
    `utils/hf_dataset_utilities.py:31-55`). Unlike the reference's closure class (which is why
    `03a…:80-97` re-defines it inline), the class is registered on this module under a name derived
    from the column names, and the module resolves such names on demand (``__getattr__``), so the
    class and its instances go through the standard pickler -- into spawn-started DataLoader workers
    and launcher children that never called this function."""
    name = _class_name(image_key, label_key)
    cls = _CLASSES.get(name)
    if cls is None:
        def __init__(self, data, transform=None):
            HFImageDataset.__init__(self, data, transform, image_key, label_key)
        cls = type(name, (HFImageDataset,), {"__init__": __init__, "__module__": __name__, "__qualname__": name,
                                             "image_key": image_key, "label_key": label_key})
        _CLASSES[name] = cls
        globals()[name] = cls
    return cls


def __getattr__(name: str):
    """PEP 562: unpickling a dataset class (or instance) in a fresh process recreates the class."""
    if name.startswith(_PREFIX):
        try:
            ih, lh = name[len(_PREFIX):].split("__")
            return create_torch_image_dataset(bytes.fromhex(ih).decode(), bytes.fromhex(lh).decode())
        except ValueError:
            pass
    raise AttributeError(f"module {__name__!r} has no attribute {name!r}")
