#!/usr/bin/env python3
"""Ray-style TorchTrainer: ResNet-18 with a 1-channel stem on FashionMNIST
(reference `05_ray/01_fashion_mnist_pytorch_ray.ipynb:167-262`): per-epoch ``report(metrics,
checkpoint=Checkpoint.from_directory(...))`` with a DDP-unwrapped ``model.pt``; the result's
checkpoint is reloaded at the end (`:308-314`)."""
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _common as C  # noqa: E402


def train_func(config):
    import torch
    import torch.nn as nn
    from torch.utils.data import DataLoader
    from dbx_distributed_pytorch_examples_amd.frontends import ray as rt
    from dbx_distributed_pytorch_examples_amd.models import resnet18_1ch
    from dbx_distributed_pytorch_examples_amd.utils.checkpoint import save_ray_checkpoint
    tr = config["train"]
    model = rt.prepare_model(resnet18_1ch(10))
    loader = rt.prepare_data_loader(DataLoader(tr, batch_size=config["batch_size"], shuffle=True))
    opt = torch.optim.Adam(model.parameters(), lr=config["lr"])
    crit = nn.CrossEntropyLoss()
    for epoch in range(config["epochs"]):
        tot, n = 0.0, 0
        for x, y in loader:
            loss = crit(model(x), y)
            opt.zero_grad()
            loss.backward()
            if hasattr(model, "finish_gradient_sync"):
                model.finish_gradient_sync()
            opt.step()
            tot, n = tot + loss.item() * y.shape[0], n + y.shape[0]
        d = tempfile.mkdtemp()
        save_ray_checkpoint(d, model)
        rt.report({"loss": tot / max(1, n), "epoch": epoch}, checkpoint=rt.Checkpoint.from_directory(d))


def main():
    args = C.parser(__doc__, procs=1, epochs=1, batch=64).parse_args()
    use_gpu = C.setup_env(args)
    import torch
    from dbx_distributed_pytorch_examples_amd.data.transforms import mnist_transforms
    from dbx_distributed_pytorch_examples_amd.frontends import ray as rt
    tr, _ = C.datasets("fashion_mnist", args, transform=mnist_transforms(fashion=True))
    rt.setup_ray_cluster(max_worker_nodes=1)
    res = rt.TorchTrainer(train_func, train_loop_config={"train": tr, "batch_size": args.batch_size, "lr": 1e-3,
                                                         "epochs": args.epochs},
                          scaling_config=rt.ScalingConfig(num_workers=args.procs, use_gpu=use_gpu),
                          run_config=rt.RunConfig(storage_path=os.path.join(args.out, "ray"), name="local")).fit()
    print("metrics:", res.metrics, "error:", res.error)
    with res.checkpoint.as_directory() as d:
        sd = torch.load(os.path.join(d, "model.pt"), weights_only=True)
    print("checkpoint tensors:", len(sd))
    rt.shutdown_ray_cluster()


if __name__ == "__main__":
    main()
