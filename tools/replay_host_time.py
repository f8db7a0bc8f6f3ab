#!/usr/bin/env python3
"""Is a graph-replayed step bound by the host's enqueue of the graph? Measures, for a bench preset:

* the host time of one ``step()`` call (the graph launch: the runtime walks the graph and writes
  every node's packets, waits and signals into the hardware queues) against the GPU time per step;
* the GPU time of one step measured with events when the GPU is held busy (``torch.cuda._sleep``)
  while the host enqueues it -- every node is already queued when the step starts -- against the
  GPU time of a step launched onto an idle GPU.

If the host time per launch approaches the GPU step time, or the pre-queued step is faster, the
step's kernels wait for the host (and a kernel trace's side-queue start times say when the host
reached the side branches, not when their dependencies were met).

  python tools/replay_host_time.py [--preset resnet50_tiny_imagenet] [--steps 20]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="resnet50_tiny_imagenet")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--sleep-cycles", type=int, default=200_000_000)
    a = ap.parse_args()
    import bench
    from dbx_distributed_pytorch_examples_amd.parallel import dist as ddist
    from dbx_distributed_pytorch_examples_amd.train.bench_steps import build_step
    args = bench.parse_args(["--preset", a.preset] if a.preset else [])
    info = ddist.init_distributed()
    step, _ = build_step(args, info)
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    # back-to-back: host time per launch and GPU time per step
    host = []
    t0 = time.perf_counter()
    for _ in range(a.steps):
        h = time.perf_counter()
        step()
        host.append(time.perf_counter() - h)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / a.steps
    host.sort()
    print(f"{a.preset or 'headline'}: back-to-back {wall * 1e3:.3f} ms/step; host per launch median "
          f"{host[len(host) // 2] * 1e3:.3f} ms, max {host[-1] * 1e3:.3f} ms")
    # one step on an idle GPU vs one step queued behind a sleep kernel (events bracket the step only)
    res = {}
    for mode in ("idle", "prequeued"):
        ts = []
        for _ in range(a.steps):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            if mode == "prequeued":
                torch.cuda._sleep(a.sleep_cycles)
            e0.record()
            step()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        ts.sort()
        res[mode] = ts[len(ts) // 2]
    print(f"  GPU step time (event, median): idle launch {res['idle']:.3f} ms, pre-queued {res['prequeued']:.3f} ms")


if __name__ == "__main__":
    main()
