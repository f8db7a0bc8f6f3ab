#!/usr/bin/env python3
"""TinyImageNet + frozen ResNet-50 with DeepSpeed-style config and early stopping
(reference `02_deepspeed/02_tiny_imagenet_deepspeed_resnet.py`, patience `:289-297`, here
rank-consistent: the stop decision is broadcast instead of breaking on rank 0 only)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _common as C  # noqa: E402


def main():
    args = C.parser(__doc__, procs=2, epochs=2, batch=32).parse_args()
    use_gpu = C.setup_env(args)
    from dbx_distributed_pytorch_examples_amd.data.transforms import default_image_transforms
    from dbx_distributed_pytorch_examples_amd.frontends import deepspeed as ds
    tr, te = C.datasets("tiny_imagenet", args, transform=default_image_transforms(64))
    dist = ds.DeepspeedTorchDistributor(numGpus=args.procs, nnodes=1, localMode=True, useGpu=use_gpu)
    model = dist.run(ds.train_func, train_dataset=tr, test_dataset=te, batch_size=args.batch_size,
                     num_epochs=args.epochs, patience=3, arch="resnet50", learning_rate=1e-3,
                     deepspeed_config=ds.deepspeed_zero_2)
    print("trained:", type(model).__name__)


if __name__ == "__main__":
    main()
