#!/usr/bin/env python3
"""Accelerate-style loop: ResNet-50 fully trainable on CIFAR-10 (reference `04_accelerate/01_cifar_accelerate.ipynb`).

Adam 1e-3 / wd 1e-4, CosineAnnealingLR(T_max=epochs) stepped per epoch, and the notebook's
``train_model(run_id) -> (history, run_id)`` (``frontends.accelerate.train_model``): metrics
train_loss / train_accuracy / test_loss / test_accuracy / learning_rate, per-epoch checkpoint dict
logged as a state dict, ``best_model`` + metadata.json, ``training_history.json``, run id broadcast
from rank 0 (`:553-790`). Launch with ``python -m
dbx_distributed_pytorch_examples_amd.launch --nproc-per-node N examples/04_accelerate/01_cifar_accelerate.py``.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _common as C  # noqa: E402


def main():
    ap = C.parser(__doc__, procs=1, epochs=1, batch=32)
    ap.add_argument("--native", action="store_true",
                    help="run this loop on the HIP kernels: engine.native_module (GPU; 2.6x at b128, profiles/r2s5_native_module)")
    args = ap.parse_args()
    use_gpu = C.setup_env(args)
    import torch
    import torch.nn as nn
    from torch.utils.data import DataLoader
    from dbx_distributed_pytorch_examples_amd.data.transforms import cifar_transforms
    from dbx_distributed_pytorch_examples_amd.frontends.accelerate import Accelerator, set_seed, train_model
    from dbx_distributed_pytorch_examples_amd.models import build_model
    from dbx_distributed_pytorch_examples_amd.parallel.sampler import ShardSampler
    config = {"batch_size": args.batch_size, "num_epochs": args.epochs, "learning_rate": 1e-3, "weight_decay": 1e-4,
              "num_classes": 10, "save_every": 1, "experiment_name": "resnet50_cifar10"}
    set_seed(42)
    acc = Accelerator(log_with="mlflow", cpu=not use_gpu)
    tr, te = C.datasets("cifar10", args, transform=cifar_transforms(True), test_transform=cifar_transforms(False))
    train_loader = DataLoader(tr, batch_size=config["batch_size"], sampler=ShardSampler(tr), pin_memory=use_gpu)
    test_loader = DataLoader(te, batch_size=config["batch_size"], sampler=ShardSampler(te, shuffle=False))
    model = build_model("resnet50", num_classes=config["num_classes"])
    if args.native and use_gpu:
        # the same loop, forward / backward on the native program (build it BEFORE the optimizer:
        # the parameters become views of the program's flat master)
        from dbx_distributed_pytorch_examples_amd.engine.native_module import native_module
        model = native_module(model, config["batch_size"], (32, 32), acc.device)
    optimizer = torch.optim.Adam(model.parameters(), lr=config["learning_rate"], weight_decay=config["weight_decay"])
    scheduler = torch.optim.lr_scheduler.CosineAnnealingLR(optimizer, T_max=config["num_epochs"])
    criterion = nn.CrossEntropyLoss()
    model, optimizer, train_loader, test_loader = acc.prepare(model, optimizer, train_loader, test_loader)
    history, run_id = train_model(None, accelerator=acc, model=model, optimizer=optimizer, scheduler=scheduler,
                                  criterion=criterion, train_loader=train_loader, test_loader=test_loader,
                                  config=config)
    if acc.is_main_process:
        print(json.dumps({"run_id": run_id, "best_test_acc": max(history["test_acc"], default=0.0)}))


if __name__ == "__main__":
    main()
