#!/usr/bin/env python3
"""TinyImageNet through MDS shards (reference `01_torch_distributor/03a_tiny_imagenet_torch_distributor_resnet_mds.py`).

Writes ``{'image': 'pil', 'label': 'int'}`` MDS shards (`:179-223`; the C++ reader in
``csrc/runtime/mds_loader.cpp`` mmaps them), then trains with ``train_func_mds`` where every rank
streams its own partition (`:346-515`) and evaluates per epoch.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _common as C  # noqa: E402


def main():
    args = C.parser(__doc__, procs=2, epochs=1, batch=32).parse_args()
    use_gpu = C.setup_env(args)
    from dbx_distributed_pytorch_examples_amd.data.mds import write_image_dataset_mds
    from dbx_distributed_pytorch_examples_amd.frontends import torch_distributor as td
    tr, te = C.datasets("tiny_imagenet", args)
    root = os.path.join(args.out, "mds_tiny_imagenet")
    for split, ds in (("train", tr), ("test", te)):
        write_image_dataset_mds(ds, os.path.join(root, split))
    print("MDS shards:", sorted(os.listdir(os.path.join(root, "train")))[:4], "...")
    model = td.TorchDistributor(num_processes=args.procs, local_mode=True, use_gpu=use_gpu).run(
        td.train_func_mds, batch_size=args.batch_size, epochs=args.epochs,
        remote=os.path.join(root, "train"), remote_val=os.path.join(root, "test"), num_classes=200)
    print("done:", type(model).__name__)


if __name__ == "__main__":
    main()
