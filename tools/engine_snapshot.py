#!/usr/bin/env python3
"""Print the step schedule the engine resolves for each step-size class: every scalar switch of
``ResNetProgram`` / ``NativeTrainer`` after the EngineConfig policy ran (single-GPU step and the
multi-rank segmented step). Runs on the CPU with a small batch and the forward-FLOP count of each
preset substituted, so it answers "what does the headline / TinyImageNet / CIFAR step run with"
without a GPU; also used to check that a refactor of the policy keeps every default.

  python tools/engine_snapshot.py [--json out.json]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# forward conv FLOPs of one step of each preset (the class the policy puts it in)
PRESET_FLOPS = {"resnet18_cifar10": ("resnet18", 2.0e10), "resnet50_tiny_imagenet": ("resnet50", 3.5e11),
                "headline": ("resnet50", 8.4e12)}
SKIP = {"model", "dev", "N", "H", "W", "training"}


def scalars(obj):
    out = {}
    for k, v in sorted(vars(obj).items()):
        if k.startswith("__") or k in SKIP:
            continue
        if isinstance(v, (bool, int, float, str)) or v is None:
            out[k] = v
    return out


def snapshot(name, arch, flops, multirank):
    import torch
    from dbx_distributed_pytorch_examples_amd.engine import program as P
    from dbx_distributed_pytorch_examples_amd.engine.native_trainer import NativeTrainer, OptimConfig
    from dbx_distributed_pytorch_examples_amd.models import build_model
    orig = P.ResNetProgram.fwd_conv_flops
    P.ResNetProgram.fwd_conv_flops = lambda self: flops
    try:
        torch.manual_seed(0)
        m = build_model(arch, num_classes=10)
        tr = NativeTrainer(m, 2, (32, 32), torch.device("cpu"), optim=OptimConfig(lr=0.1), use_graphs=False)
        d = {"program": scalars(tr.prog), "trainer": {k: v for k, v in scalars(tr).items()
                                                      if k not in ("step_count", "world")}}
    finally:
        P.ResNetProgram.fwd_conv_flops = orig
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    import torch.distributed as dist
    res = {}
    for name, (arch, fl) in PRESET_FLOPS.items():
        res[name] = snapshot(name, arch, fl, False)
    # the multi-rank layout: a one-rank gloo group with the segmented step forced
    import tempfile
    with tempfile.TemporaryDirectory() as td:
        dist.init_process_group("gloo", init_method=f"file://{td}/pg", rank=0, world_size=1)
        os.environ["DBX_ENGINE"] = ",".join(s for s in (os.environ.get("DBX_ENGINE", ""), "segmented_graphs=1") if s)
        try:
            for name, (arch, fl) in PRESET_FLOPS.items():
                res[name + "@segmented"] = snapshot(name, arch, fl, True)
        finally:
            dist.destroy_process_group()
    txt = json.dumps(res, indent=1, sort_keys=True)
    if a.json:
        with open(a.json, "w") as f:
            f.write(txt)
    else:
        print(txt)


if __name__ == "__main__":
    main()
