#!/usr/bin/env python3
"""ImageNet-1K 224x224 + frozen ResNet-50 (reference `02_deepspeed/03_1k_imagenet_deepspeed_resnet.py`).

The reference calls ``dist.run(train_func, epochs=...)`` although the function takes
``num_epochs`` (a TypeError); this script passes ``num_epochs``. Transforms:
RandomResizedCrop(224) + flip for train, Resize+CenterCrop for eval (the reference reuses the
training crop for validation)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _common as C  # noqa: E402


def main():
    args = C.parser(__doc__, procs=2, epochs=1, batch=16).parse_args()
    args.samples = min(args.samples, 128)
    use_gpu = C.setup_env(args)
    from dbx_distributed_pytorch_examples_amd.data.transforms import imagenet_transforms
    from dbx_distributed_pytorch_examples_amd.frontends import deepspeed as ds
    tr, te = C.datasets("imagenet", args, transform=imagenet_transforms(True), test_transform=imagenet_transforms(False))
    dist = ds.DeepspeedTorchDistributor(numGpus=args.procs, nnodes=1, localMode=True, useGpu=use_gpu)
    model = dist.run(ds.train_func, train_dataset=tr, test_dataset=te, batch_size=args.batch_size,
                     num_epochs=args.epochs, arch="resnet50", deepspeed_config=ds.deepspeed_zero_1)
    print("trained:", type(model).__name__)


if __name__ == "__main__":
    main()
