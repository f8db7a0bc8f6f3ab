#!/usr/bin/env python3
"""TinyImageNet (64x64, 200 classes) + frozen ResNet-50 with TorchDistributor
(reference `01_torch_distributor/03_tiny_imagenet_torch_distributor_resnet.py`)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _common as C  # noqa: E402


def main():
    args = C.parser(__doc__, procs=2, epochs=1, batch=32).parse_args()
    use_gpu = C.setup_env(args)
    from dbx_distributed_pytorch_examples_amd.data.transforms import default_image_transforms
    from dbx_distributed_pytorch_examples_amd.frontends import torch_distributor as td
    tr, te = C.datasets("tiny_imagenet", args, transform=default_image_transforms(64))
    model = td.TorchDistributor(num_processes=args.procs, local_mode=True, use_gpu=use_gpu).run(
        td.train_func, train_dataset=tr, test_dataset=te, batch_size=args.batch_size, epochs=args.epochs,
        arch="resnet50")
    print(type(model).__name__, sum(p.numel() for p in model.parameters() if p.requires_grad), "trainable params")


if __name__ == "__main__":
    main()
