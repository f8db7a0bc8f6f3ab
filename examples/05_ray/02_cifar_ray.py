#!/usr/bin/env python3
"""Ray-style TorchTrainer: random-init ResNet-18 on CIFAR-10 (reference `05_ray/02_cifar_resnet_pytorch_ray.ipynb`),
Adam 1e-5, batch 256 in the notebook; the dataset is handed to workers through the loop config
(the notebook captures it in a closure)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _common as C  # noqa: E402


def train_func(config):
    import torch
    import torch.nn as nn
    from torch.utils.data import DataLoader
    from dbx_distributed_pytorch_examples_amd.frontends import ray as rt
    from dbx_distributed_pytorch_examples_amd.models import build_model
    # --native: the worker's loop on the HIP kernels (engine.native_module via prepare_model)
    model = rt.prepare_model(build_model("resnet18", num_classes=10),
                             native_batch=config["batch_size"] if config.get("native") else 0, native_hw=(32, 32))
    loader = rt.prepare_data_loader(DataLoader(config["train"], batch_size=config["batch_size"], shuffle=True))
    opt = torch.optim.Adam(model.parameters(), lr=config["lr"])
    for epoch in range(config["epochs"]):
        tot, n, corr = 0.0, 0, 0
        for x, y in loader:
            out = model(x)
            loss = nn.functional.cross_entropy(out, y)
            opt.zero_grad()
            loss.backward()
            if hasattr(model, "finish_gradient_sync"):
                model.finish_gradient_sync()
            opt.step()
            tot, n, corr = tot + loss.item() * y.shape[0], n + y.shape[0], corr + int((out.argmax(1) == y).sum())
        rt.report({"loss": tot / max(1, n), "accuracy": corr / max(1, n), "epoch": epoch})


def main():
    ap = C.parser(__doc__, procs=1, epochs=1, batch=64)
    ap.add_argument("--native", action="store_true", help="GPU: the loop on engine.native_module")
    args = ap.parse_args()
    use_gpu = C.setup_env(args)
    from dbx_distributed_pytorch_examples_amd.data.transforms import default_image_transforms
    from dbx_distributed_pytorch_examples_amd.frontends import ray as rt
    tr, _ = C.datasets("cifar10", args, transform=default_image_transforms(32))
    res = rt.TorchTrainer(train_func, train_loop_config={"train": tr, "batch_size": args.batch_size, "lr": 1e-5,
                                                         "epochs": args.epochs, "native": args.native},
                          scaling_config=rt.ScalingConfig(num_workers=args.procs, use_gpu=use_gpu),
                          run_config=rt.RunConfig(storage_path=os.path.join(args.out, "ray"), name="cifar")).fit()
    print("metrics:", res.metrics, "error:", res.error)


if __name__ == "__main__":
    main()
