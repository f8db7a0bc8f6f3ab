#!/usr/bin/env python3
"""Accelerate-style loop: ResNet-50 fully trainable on CIFAR-10 (reference `04_accelerate/01_cifar_accelerate.ipynb`).

Adam 1e-3 / wd 1e-4, CosineAnnealingLR(T_max=epochs) stepped per epoch, metrics gathered across
processes, per-epoch checkpoint dict {epoch, model/optimizer/scheduler state, test_accuracy} logged
to MLflow as a state dict, best model logged as ``best_model`` + metadata.json, history JSON, and
the run id broadcast from rank 0 (`:553-790`). Launch with ``python -m
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
    from dbx_distributed_pytorch_examples_amd.frontends.accelerate import Accelerator, set_seed
    from dbx_distributed_pytorch_examples_amd.models import build_model
    from dbx_distributed_pytorch_examples_amd.parallel.sampler import ShardSampler
    from dbx_distributed_pytorch_examples_amd.utils import mlflow_compat as mlflow
    from dbx_distributed_pytorch_examples_amd.utils.checkpoint import accelerate_checkpoint
    config = {"batch_size": args.batch_size, "num_epochs": args.epochs, "learning_rate": 1e-3, "weight_decay": 1e-4,
              "num_classes": 10}
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
    run_id = None
    if acc.is_main_process:
        run_id = mlflow.start_run().info.run_id
        mlflow.log_params({**config, "optimizer": "Adam", "scheduler": "CosineAnnealingLR",
                           "num_gpus": acc.num_processes})
    history, best = {"train_loss": [], "train_acc": [], "test_loss": [], "test_acc": [], "lr": []}, 0.0
    for epoch in range(config["num_epochs"]):
        model.train()
        sums = torch.zeros(3, device=acc.device)
        for x, y in train_loader:
            optimizer.zero_grad()
            with acc.autocast():
                out = model(x)
                loss = criterion(out.float(), y)
            acc.backward(loss)
            optimizer.step()
            sums += torch.stack([loss.detach() * y.shape[0], (out.argmax(1) == y).sum().float(),
                                 torch.tensor(float(y.shape[0]), device=sums.device)])
        tl, tc, tn = acc.reduce(sums).tolist()
        model.eval()
        ev = torch.zeros(3, device=acc.device)
        with torch.no_grad():
            for x, y in test_loader:
                with acc.autocast():
                    out = model(x)
                ev += torch.stack([criterion(out.float(), y) * y.shape[0], (out.argmax(1) == y).sum().float(),
                                   torch.tensor(float(y.shape[0]), device=ev.device)])
        el, ec, en = acc.reduce(ev).tolist()
        lr = scheduler.get_last_lr()[0]
        scheduler.step()
        if acc.is_main_process:
            rec = {"train_loss": tl / tn, "train_acc": 100 * tc / tn, "test_loss": el / en, "test_acc": 100 * ec / en,
                   "lr": lr}
            for k, v in rec.items():
                history[k].append(v)
            mlflow.log_metrics(rec, step=epoch)
            ck = accelerate_checkpoint(epoch + 1, acc.unwrap_model(model), optimizer, scheduler, rec["test_acc"])
            mlflow.pytorch.log_state_dict(ck, f"checkpoints/epoch_{epoch + 1}")
            if rec["test_acc"] >= best:
                best = rec["test_acc"]
                mlflow.pytorch.log_model(acc.unwrap_model(model), "best_model")
                mlflow.log_dict({"epoch": epoch + 1, "test_accuracy": best}, "best_model/metadata.json")
            print(f"epoch {epoch + 1}: {rec}")
        acc.wait_for_everyone()
    if acc.is_main_process:
        mlflow.log_dict(history, "history.json")
        mlflow.end_run()
        print(json.dumps({"run_id": run_id, "best_test_acc": best}))


if __name__ == "__main__":
    main()
