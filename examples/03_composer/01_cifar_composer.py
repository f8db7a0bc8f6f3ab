#!/usr/bin/env python3
"""Composer-style training of a random-init ResNet-50 on CIFAR-10
(reference `03_composer/01_cifar_composer_resnet.ipynb:406-436`): Adam 1e-4, batch 128,
``max_duration="2ep"``, algorithms LabelSmoothing(0.1) + CutMix(1.0) + ChannelsLast, MLflow logger."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _common as C  # noqa: E402


def main():
    ap = C.parser(__doc__, procs=1, epochs=1, batch=32)
    ap.add_argument("--duration", default="")
    args = ap.parse_args()
    use_gpu = C.setup_env(args)
    import torch
    from torch.utils.data import DataLoader
    from dbx_distributed_pytorch_examples_amd.data.transforms import cifar_transforms
    from dbx_distributed_pytorch_examples_amd.frontends import composer as cp
    from dbx_distributed_pytorch_examples_amd.models import ComposerResNet50
    from dbx_distributed_pytorch_examples_amd.utils.inference import predict_image
    tr, te = C.datasets("cifar10", args, transform=cifar_transforms(True), test_transform=cifar_transforms(False))
    model = ComposerResNet50(num_classes=1000)  # the notebook keeps the 1000-way head
    trainer = cp.Trainer(model=model, optimizers=torch.optim.Adam(model.parameters(), lr=1e-4),
                         train_dataloader=DataLoader(tr, batch_size=args.batch_size, shuffle=True),
                         eval_dataloader=DataLoader(te, batch_size=args.batch_size),
                         max_duration=args.duration or f"{args.epochs}ep",
                         algorithms=[cp.LabelSmoothing(0.1), cp.CutMix(alpha=1.0, num_classes=1000), cp.ChannelsLast()],
                         loggers=[cp.MLFlowLogger(experiment_name="composer_cifar")],
                         device="cuda" if use_gpu else "cpu")
    import time
    t0 = time.time()
    hist = trainer.fit()
    print(f"fit: {time.time() - t0:.1f}s ({'native HIP program' if trainer.native else 'torch module'})")
    print(hist[-1])
    img, label = C.datasets("cifar10", args)[1][0]
    # (on the GPU the native module's parameters stay on the device: predict there)
    dev = "cuda" if use_gpu else "cpu"
    predict_image(trainer.model if use_gpu else trainer.model.cpu(), img, device=dev, true_label=label)
    trainer.close()


if __name__ == "__main__":
    main()
