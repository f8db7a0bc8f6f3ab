"""Shared helpers for the example scripts: repo import path, offline datasets, CLI flags.

The reference notebooks download CIFAR-10 / TinyImageNet / ImageNet-1K / MNIST from Hugging Face or
torchvision. This node is offline, so every example defaults to synthetic data of the same shape
(uint8 HWC images + labels); pass ``--data-root`` to use real local copies (CIFAR-10 binary batches,
MNIST IDX files, an ImageFolder tree, or an MDS directory).
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

SHAPES = {  # dataset -> (image size, channels, classes)
    "cifar10": (32, 3, 10), "tiny_imagenet": (64, 3, 200), "imagenet": (224, 3, 1000),
    "mnist": (28, 1, 10), "fashion_mnist": (28, 1, 10),
}


def parser(desc: str, procs: int = 2, epochs: int = 1, batch: int = 32) -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description=desc)
    ap.add_argument("--procs", type=int, default=procs, help="processes (one per GPU; gloo ranks on CPU)")
    ap.add_argument("--epochs", type=int, default=epochs)
    ap.add_argument("--batch-size", type=int, default=batch)
    ap.add_argument("--samples", type=int, default=256, help="synthetic samples per split")
    ap.add_argument("--data-root", default="", help="real dataset location (default: synthetic)")
    ap.add_argument("--cpu", action="store_true", help="force CPU/gloo even if GPUs are present")
    ap.add_argument("--out", default=os.path.join(ROOT, "runs"), help="checkpoints / mlruns root")
    return ap


def setup_env(args) -> bool:
    """Returns use_gpu. Points MLflow at a local file store under --out."""
    os.makedirs(args.out, exist_ok=True)
    os.environ.setdefault("DBX_MLRUNS", os.path.join(args.out, "mlruns"))
    if args.cpu:
        os.environ["DBX_FORCE_CPU"] = "1"
    try:
        import torch
        return (not args.cpu) and torch.cuda.device_count() > 0
    except Exception:
        return False


def datasets(name: str, args, transform=None, test_transform=None):
    """(train, test) datasets: real ones from --data-root, else synthetic of the right shape."""
    from dbx_distributed_pytorch_examples_amd.data.datasets import SyntheticImages, build_dataset
    size, ch, classes = SHAPES[name]
    if args.data_root:
        tr = build_dataset(name, args.data_root, True, transform, size, classes)
        te = build_dataset(name, args.data_root, False, test_transform or transform, size, classes)
        return tr, te
    tr = SyntheticImages(args.samples, size, ch, classes, seed=1, transform=transform)
    te = SyntheticImages(max(64, args.samples // 4), size, ch, classes, seed=2, transform=test_transform or transform)
    tr.num_classes = te.num_classes = classes
    return tr, te
