"""Command-line training: ``python -m dbx_distributed_pytorch_examples_amd.train.cli CONFIG [k=v ...]``.

One process per GPU: launch with ``python -m dbx_distributed_pytorch_examples_amd.launch
--nproc-per-node 8 -m dbx_distributed_pytorch_examples_amd.train.cli CONFIG`` or ``torchrun`` (env:// rendezvous, RCCL). ``--deepspeed FILE`` maps a
DeepSpeed JSON/YAML (the reference's `02_deepspeed/deepspeed_config.py` schema) onto the config.
Prints one JSON summary line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import sys

import yaml

from ..config import from_deepspeed, load_config, to_dict
from .engine import train


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("config", nargs="?", default=None, help="YAML/JSON TrainConfig (configs/*.yaml)")
    ap.add_argument("overrides", nargs="*", help="dotted overrides, e.g. optim.lr=0.2 data.dataset=synthetic")
    ap.add_argument("--deepspeed", default=None, help="DeepSpeed config file applied on top")
    ap.add_argument("--print-config", action="store_true")
    a = ap.parse_args(argv)
    cfg = load_config(a.config, a.overrides)
    if a.deepspeed:
        with open(a.deepspeed) as f:
            cfg = from_deepspeed(yaml.safe_load(f), cfg)
    if a.print_config:
        print(json.dumps(to_dict(cfg), indent=1, default=str))
        return 0
    res = train(cfg)
    from ..parallel import dist as ddist
    if ddist.get_rank() == 0:
        last = res.history[-1] if res.history else {}
        print(json.dumps({"engine": res.engine, "steps": res.steps, "images_per_sec": round(res.images_per_sec, 2),
                          "best_val_accuracy": res.best_val_accuracy, "run_id": res.run_id, **last}, default=float))
    return 0


if __name__ == "__main__":
    sys.exit(main())
