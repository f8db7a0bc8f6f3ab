#!/usr/bin/env python3
"""CIFAR-10 + frozen ResNet-18 head training with TorchDistributor
(reference `01_torch_distributor/02_cifar_torch_distributor_resnet.py`).

``train_func(train_dataset=..., test_dataset=..., batch_size, epochs)`` keeps the notebook's
signature (`:165-304`) but the N processes form ONE data-parallel job (the reference's ranks never
join a process group and train N independent replicas). Ends with the notebook's single-image
prediction (`:366-387`) — normalised here (the reference forgets Normalize at inference).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _common as C  # noqa: E402


def main():
    ap = C.parser(__doc__, procs=2, epochs=1, batch=64)
    ap.add_argument("--arch", default="resnet18")
    args = ap.parse_args()
    use_gpu = C.setup_env(args)
    from dbx_distributed_pytorch_examples_amd.data.transforms import default_image_transforms
    from dbx_distributed_pytorch_examples_amd.frontends import torch_distributor as td
    from dbx_distributed_pytorch_examples_amd.utils.inference import predict_image
    from dbx_distributed_pytorch_examples_amd.utils.timer import Timer
    tf = default_image_transforms(32)
    tr, te = C.datasets("cifar10", args, transform=tf)
    timer = Timer()
    model = td.TorchDistributor(num_processes=args.procs, local_mode=True, use_gpu=use_gpu).run(
        td.train_func, train_dataset=tr, test_dataset=te, batch_size=args.batch_size, epochs=args.epochs)
    print(f"trained in {timer.stop():.1f}s")
    img, label = C.datasets("cifar10", args)[1][0]
    predict_image(model.cpu(), img, device="cpu", true_label=label)


if __name__ == "__main__":
    main()
