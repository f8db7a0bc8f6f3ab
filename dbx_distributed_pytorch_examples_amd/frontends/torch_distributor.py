"""TorchDistributor-style entrypoints (`01_torch_distributor/*.py`) on the native stack.

Reference functions, same names / signatures, real data parallelism:

* MNIST: ``train_one_epoch``, ``train(log_dir)``, ``test(log_dir)`` (`01_basic_torch_distributor.py:93-181`)
  and ``main_fn(directory)`` (`:248-328`: process group, ShardSampler, DDP, rank-0 checkpoint /
  log / eval) — run with ``TorchDistributor(num_processes=N, local_mode=True).run(main_fn, dir)``;
  on a GPU the ``Net`` trains on the fused HIP kernels (``engine.native_mnist``);
* ResNet: ``train_func(*, train_dataset, test_dataset, batch_size=32, epochs=5, mlflow_run_id=None)``
  (`02_cifar_torch_distributor_resnet.py:165-304`, `03_tiny_imagenet…:149-288`). The reference's
  version never forms a process group (each rank trains an independent replica);
  here the ranks are one data-parallel job via ``train.engine.train``;
* MDS: ``train_func_mds(*, batch_size=128, epochs=5, mlflow_run_id=None, patience=4, remote=…, local=…)``
  (`03a_tiny_imagenet_torch_distributor_resnet_mds.py:346-515`).
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.nn.functional as F
from torch.utils.data import DataLoader

from ..config import TrainConfig
from ..launch import TorchDistributor  # noqa: F401  (re-export)
from ..models import FrozenBackboneClassifier, Net, build_model
from ..parallel import dist as ddist
from ..parallel.ddp import DistributedDataParallel
from ..parallel.sampler import ShardSampler
from ..train.engine import train as _train
from ..utils import mlflow_compat as mlflow
from ..utils.checkpoint import create_log_dir, load_checkpoint, save_checkpoint  # noqa: F401

batch_size = 100
num_epochs = 10
momentum = 0.5
log_interval = 100
learning_rate = 0.001


def train_one_epoch(model, device, data_loader, optimizer, epoch, log_interval: int = log_interval):
    model.train()
    for batch_idx, (data, target) in enumerate(data_loader):
        data, target = data.to(device), target.to(device)
        optimizer.zero_grad()
        loss = F.nll_loss(model(data), target)
        loss.backward()
        if hasattr(model, "finish_gradient_sync"):
            model.finish_gradient_sync()
        optimizer.step()
        if batch_idx % log_interval == 0:
            print(f"Train Epoch: {epoch} [{batch_idx * len(data)}/{len(data_loader.dataset)}]\tLoss: {loss.item():.6f}")
            if ddist.get_rank() == 0 and mlflow.active_run() is not None:
                mlflow.log_metric("train_loss", loss.item())


def _mnist(train: bool, dataset=None):
    if dataset is not None:
        return dataset
    from ..data.datasets import MNIST, SyntheticImages
    from ..data.transforms import mnist_transforms
    root = os.environ.get("DBX_MNIST_ROOT", "data")
    try:
        return MNIST(root, train=train, transform=mnist_transforms())
    except FileNotFoundError:
        # no download on this image: synthetic 28x28 digits-shaped data keeps the examples runnable
        return SyntheticImages(600 if train else 100, 28, 1, 10, seed=int(train), transform=mnist_transforms())


def train(log_dir: str, dataset=None, epochs: int = num_epochs, device: Optional[str] = None):
    """Single-process MNIST training (`01_basic…:134-153`); checkpoints every epoch."""
    dev = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
    from ..engine.native_mnist import native_mnist
    model = native_mnist(Net(), dev)  # GPU: the fused HIP Net (csrc/mnist_ops.hip); CPU: the module
    loader = DataLoader(_mnist(True, dataset), batch_size=batch_size, shuffle=True)
    opt = torch.optim.SGD(model.parameters(), lr=learning_rate, momentum=momentum)
    for epoch in range(1, epochs + 1):
        train_one_epoch(model, dev, loader, opt, epoch)
        save_checkpoint(log_dir, model, opt, epoch)
    return getattr(model, "module", model)


def test(log_dir: str, dataset=None, epoch: int = num_epochs, device: Optional[str] = None) -> float:
    """Load ``checkpoint-{epoch}`` and report mean test NLL (`01_basic…:155-181`)."""
    dev = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
    st = load_checkpoint(log_dir, epoch)
    model = Net().to(dev)
    model.load_state_dict(st["model"])
    model.eval()
    loader = DataLoader(_mnist(False, dataset), batch_size=256)
    loss, n = 0.0, 0
    with torch.no_grad():
        for x, y in loader:
            out = model(x.to(dev))
            loss += F.nll_loss(out, y.to(dev), reduction="sum").item()
            n += y.shape[0]
    test_loss = loss / max(1, n)
    print(f"Average test loss: {test_loss}")
    if mlflow.active_run() is not None:
        mlflow.log_metric("test_loss", test_loss)
    return test_loss


def main_fn(directory: str, train_dataset=None, test_dataset=None, epochs: int = num_epochs):
    """DDP MNIST (`01_basic…:248-328`): one process per GPU (or gloo ranks on CPU)."""
    info = ddist.init_distributed(device="cpu" if os.environ.get("DBX_FORCE_CPU") == "1" else None)
    rank = info.rank
    if rank == 0 and mlflow.active_run() is None:
        mlflow.start_run()
        mlflow.log_params({"batch_size": batch_size, "epochs": epochs, "trainer": "TorchDistributor"})
    ds = _mnist(True, train_dataset)
    sampler = ShardSampler(ds)
    loader = DataLoader(ds, batch_size=batch_size, sampler=sampler)
    if info.device.type == "cuda":
        # the fused HIP Net: broadcasts rank 0's weights and averages its flat gradient itself (DDP semantics)
        from ..engine.native_mnist import native_mnist
        model = native_mnist(Net(), info.device)
    else:
        model = DistributedDataParallel(Net().to(info.device))
    opt = torch.optim.SGD(model.parameters(), lr=learning_rate, momentum=momentum)
    for epoch in range(1, epochs + 1):
        sampler.set_epoch(epoch)
        train_one_epoch(model, info.device, loader, opt, epoch)
        if rank == 0:
            save_checkpoint(directory, model, opt, epoch)
    if rank == 0:
        mlflow.pytorch.log_model(model, "model")
        model.module.eval()
        loss, n = 0.0, 0
        with torch.no_grad():
            for x, y in DataLoader(_mnist(False, test_dataset), batch_size=256):
                loss += F.nll_loss(model.module(x.to(info.device)), y.to(info.device), reduction="sum").item()
                n += y.shape[0]
        mlflow.log_metric("test_loss", loss / max(1, n))
        mlflow.end_run()
    ddist.barrier()
    ddist.destroy()
    return "finished"


def train_func(*, train_dataset, test_dataset, batch_size: int = 32, epochs: int = 5, mlflow_run_id=None,
               arch: str = "resnet18", frozen_backbone: bool = True, learning_rate: float = 1e-3,
               model_name: str = "cifar_torch_distributor_resnet", **cfg_kw):
    """ResNet train_func of the TD notebooks: Adam(lr), CE, per-epoch train/val metrics on rank 0; the
    model is logged as ``model_name`` (both `02_cifar_…:267` and `03_tiny_imagenet_…:251` use
    "cifar_torch_distributor_resnet")."""
    num_classes = getattr(test_dataset, "num_classes", None) or getattr(train_dataset, "num_classes", 10)
    model = (FrozenBackboneClassifier(arch, num_classes) if frozen_backbone else build_model(arch, num_classes=num_classes))
    cfg = TrainConfig(model=arch, num_classes=num_classes, batch_size=batch_size, epochs=epochs, log_every=10,
                      experiment=os.environ.get("MLFLOW_EXPERIMENT_NAME", "torch_distributor"), model_name=model_name)
    cfg.optim.name, cfg.optim.lr, cfg.optim.weight_decay = "adam", learning_rate, 0.0
    for k, v in cfg_kw.items():
        setattr(cfg, k, v)
    res = _train(cfg, model=model, train_dataset=train_dataset, eval_dataset=test_dataset,
                 log_mlflow=mlflow_run_id is not None or os.environ.get("DBX_LOG_MLFLOW") == "1")
    return res.model


def train_func_mds(*, batch_size: int = 128, epochs: int = 5, mlflow_run_id=None, patience: int = 4,
                   remote: Optional[str] = None, local: Optional[str] = None, remote_val: Optional[str] = None,
                   num_classes: int = 200, arch: str = "resnet50", image_size: int = 64, frozen_backbone: bool = True,
                   model_name: str = "cifar_torch_distributor_resnet_mds"):
    """03a: train from MDS shards (rank-partitioned StreamingDataset), per-epoch eval, early stop. As in
    the notebook (`03a_…_mds.py:321-340`) the default trains a Dropout(0.5)+Linear head on a frozen
    ResNet-50 (``frozen_backbone=False``: the whole network); logged as ``model_name`` (`:466`)."""
    from ..data.mds import StreamingDataset
    ds = StreamingDataset(remote=remote, local=local, shuffle=True, batch_size=batch_size)
    ev = StreamingDataset(remote=remote_val, local=(local + "_val") if (local and remote_val) else remote_val) \
        if remote_val else None
    model = FrozenBackboneClassifier(arch, num_classes) if frozen_backbone else build_model(arch, num_classes=num_classes)
    cfg = TrainConfig(model=arch, num_classes=num_classes, batch_size=batch_size, epochs=epochs, patience=patience,
                      experiment=os.environ.get("MLFLOW_EXPERIMENT_NAME", "torch_distributor_mds"), model_name=model_name)
    cfg.data.image_size = image_size
    cfg.data.dataset = "mds"
    cfg.optim.name, cfg.optim.lr, cfg.optim.weight_decay = "adam", 1e-3, 0.0
    res = _train(cfg, model=model, train_dataset=ds, eval_dataset=ev, log_mlflow=mlflow_run_id is not None)
    return res.model
