#!/usr/bin/env python3
"""CIFAR-10 + frozen ResNet-18 with the DeepSpeed launcher (reference `02_deepspeed/01_cifar_deepspeed_resnet.py`).

The reference builds `deepspeed_config.py` dicts but never passes them (its `:108` is commented out);
here ``deepspeedConfig=`` is applied: bf16, AdamW + WarmupLR, clipping 0.3 and ZeRO stage 1/2
optimizer-state sharding over the ranks (``parallel/zero.py``), or stage 3 parameter sharding with
optional CPU offload (``--zero 3`` / ``--zero 3-offload``, ``parallel/fsdp.py``).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _common as C  # noqa: E402


def main():
    ap = C.parser(__doc__, procs=2, epochs=1, batch=64)
    ap.add_argument("--zero", default="1", choices=["0", "1", "2", "3", "3-offload"])
    args = ap.parse_args()
    use_gpu = C.setup_env(args)
    from dbx_distributed_pytorch_examples_amd.data.transforms import default_image_transforms
    from dbx_distributed_pytorch_examples_amd.frontends import deepspeed as ds
    tr, te = C.datasets("cifar10", args, transform=default_image_transforms(32))
    cfg = {"0": ds.base_config, "1": ds.deepspeed_zero_1, "2": ds.deepspeed_zero_2, "3": ds.deepspeed_zero_3,
           "3-offload": ds.deepspeed_zero_3_offload}[args.zero]
    dist = ds.DeepspeedTorchDistributor(numGpus=args.procs, nnodes=1, localMode=True, useGpu=use_gpu,
                                        deepspeedConfig=cfg)
    model = dist.run(ds.train_func, train_dataset=tr, test_dataset=te, batch_size=args.batch_size,
                     num_epochs=args.epochs, deepspeed_config=cfg)
    print("trained:", type(model).__name__)


if __name__ == "__main__":
    main()
