#!/usr/bin/env python3
"""MNIST with TorchDistributor (reference `01_torch_distributor/01_basic_torch_distributor.py`).

Three stages like the notebook: single-process ``train``/``test`` (`:134-181`), then ``main_fn`` as
real DDP over N processes (`:248-328`, `:357-372`): ShardSampler, flat-bucket DDP on RCCL (gloo on
CPU), rank-0 checkpoints ``checkpoint-{epoch}.pth.tar`` and evaluation.
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _common as C  # noqa: E402


def _local(log_dir, tr, te, epochs, device):
    from dbx_distributed_pytorch_examples_amd.frontends import torch_distributor as td
    td.train(log_dir, dataset=tr, epochs=epochs, device=device)
    td.test(log_dir, dataset=te, epoch=epochs, device=device)


def main():
    args = C.parser(__doc__, procs=2, epochs=1, batch=100).parse_args()
    use_gpu = C.setup_env(args)
    from dbx_distributed_pytorch_examples_amd.data.transforms import mnist_transforms
    from dbx_distributed_pytorch_examples_amd.frontends import torch_distributor as td
    from dbx_distributed_pytorch_examples_amd.utils.checkpoint import create_log_dir
    tr, te = C.datasets("mnist", args, transform=mnist_transforms())
    # single process (the notebook's "local" section)
    log_dir = create_log_dir(os.path.join(args.out, "mnist_local"))
    t = time.time()
    if use_gpu:
        # on the GPU the local section runs in ONE child process: this process must not initialise the
        # GPU before it spawns the distributed ranks below (the launcher refuses to spawn from it then)
        td.TorchDistributor(num_processes=1, local_mode=True, use_gpu=True).run(_local, log_dir, tr, te, args.epochs,
                                                                                 "cuda")
    else:
        _local(log_dir, tr, te, args.epochs, "cpu")
    print(f"local: {time.time() - t:.1f}s")
    # distributed (TorchDistributor(num_processes=N, local_mode=True).run(main_fn, dir))
    ddp_dir = create_log_dir(os.path.join(args.out, "mnist_ddp"))
    t = time.time()
    r = td.TorchDistributor(num_processes=args.procs, local_mode=True, use_gpu=use_gpu).run(
        td.main_fn, ddp_dir, tr, te, args.epochs)
    print(f"distributed x{args.procs}: {r} in {time.time() - t:.1f}s; checkpoints in {ddp_dir}")


if __name__ == "__main__":
    main()
