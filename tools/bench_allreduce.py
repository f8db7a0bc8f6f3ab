#!/usr/bin/env python3
"""RCCL all-reduce / reduce-scatter / all-gather bandwidth over message sizes (the DDP bucket
sizing check of SURVEY.md §7.2 step 4): algbw = bytes / time, busbw = algbw * 2(n-1)/n for
all-reduce ((n-1)/n for reduce-scatter / all-gather), as nccl-tests report them.

  python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 tools/bench_allreduce.py
  (CPU / gloo: DBX_DIST_BACKEND=gloo ... --device cpu)
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dbx_distributed_pytorch_examples_amd.parallel import dist as ddist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes-mb", default="1,4,16,25,64,102,256")
    ap.add_argument("--dtype", default="float32", choices=["float32", "bfloat16"])
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--device", default=None, help="cuda | cpu (default: cuda when available)")
    a = ap.parse_args()
    info = ddist.init_distributed(device=a.device)
    n = info.world_size
    dt = getattr(torch, a.dtype)
    esz = torch.tensor([], dtype=dt).element_size()
    sync = (lambda: torch.cuda.synchronize()) if info.device.type == "cuda" else (lambda: None)
    rows = []
    for mb in [float(s) for s in a.sizes_mb.split(",")]:
        numel = int(mb * (1 << 20) // esz) // n * n
        x = torch.ones(numel, dtype=dt, device=info.device)
        shard = torch.empty(numel // n, dtype=dt, device=info.device)
        res = {}
        for op in ("all_reduce", "reduce_scatter", "all_gather"):
            def run():
                if op == "all_reduce":
                    dist.all_reduce(x)
                elif op == "reduce_scatter":
                    dist.reduce_scatter_tensor(shard, x)
                else:
                    dist.all_gather_into_tensor(x, shard)
            for _ in range(3):
                run()
            sync()
            ddist.barrier()
            t0 = time.perf_counter()
            for _ in range(a.iters):
                run()
            sync()
            dt_s = ddist.all_reduce_max((time.perf_counter() - t0) / a.iters)
            nbytes = numel * esz
            algbw = nbytes / dt_s / 1e9
            factor = 2 * (n - 1) / n if op == "all_reduce" else (n - 1) / n
            res[op] = {"us": round(dt_s * 1e6, 1), "algbw_GBps": round(algbw, 1), "busbw_GBps": round(algbw * factor, 1)}
        rows.append({"size_mb": mb, **res})
        if info.rank == 0:
            print(json.dumps({"size_mb": mb, **res}), flush=True)
    if info.rank == 0:
        print(json.dumps({"world": n, "backend": info.backend, "dtype": a.dtype, "results": rows}))
    ddist.destroy()


if __name__ == "__main__":
    main()
