#!/usr/bin/env python3
"""Minimal reproducer hunt for the hipGraphLaunch SIGSEGV behind the package's
``DEBUG_HIP_FORCE_GRAPH_QUEUES=2`` default (profiles/r4_final2/README.md: the runtime's per-branch
stream assignment reads past its stream pool when pool entries equal to the launch stream are skipped).

Each case runs in a FRESH child process (the queue setting is read once, at HIP initialisation): a HIP
graph whose capture forks into B parallel branches of small kernels on B side streams (optionally
re-using the launch stream inside the capture, optionally launched on a stream that also ran eager work
before), replayed R times; the child's exit status is reported (-11 = the SIGSEGV). The parent never
touches the GPU.

  python tools/repro_graph_queues.py [--queues unset,4,2,1] [--branches 2,3,5,8] [--replays 50]
"""
import argparse
import itertools
import json
import os
import subprocess
import sys

CHILD = r"""
import sys, torch
B, R, reuse, launch_side = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3] == "1", sys.argv[4] == "1"
dev = torch.device("cuda", 0)
x = [torch.ones(1 << 16, device=dev) for _ in range(B + 1)]
side = [torch.cuda.Stream(device=dev) for _ in range(B)]
cap = side[0] if launch_side else torch.cuda.Stream(device=dev)
if launch_side:  # eager work on the stream that will also launch the graph
    with torch.cuda.stream(cap):
        x[0].mul_(1.0)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
cap.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(cap):
    with torch.cuda.graph(g, stream=cap):
        x[0].add_(1.0)
        for b in range(B):
            s = cap if (reuse and b == 0) else side[b]
            if s is not cap:
                s.wait_stream(cap)
            with torch.cuda.stream(s):
                for _ in range(3):
                    x[b + 1].mul_(1.0001)
            if s is not cap:
                cap.wait_stream(s)
        x[0].add_(1.0)
torch.cuda.synchronize()
with torch.cuda.stream(cap):
    for _ in range(R):
        g.replay()
torch.cuda.synchronize()
print("ok", float(x[0][0]))
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--queues", default="unset,4,2,1")
    ap.add_argument("--branches", default="2,3,5,8")
    ap.add_argument("--replays", type=int, default=50)
    ap.add_argument("--timeout", type=float, default=60.0)
    a = ap.parse_args()
    rows = []
    for q, b, reuse, ls in itertools.product(a.queues.split(","), [int(v) for v in a.branches.split(",")],
                                             (0, 1), (0, 1)):
        env = dict(os.environ)
        env.pop("DEBUG_HIP_FORCE_GRAPH_QUEUES", None)
        if q != "unset":
            env["DEBUG_HIP_FORCE_GRAPH_QUEUES"] = q
        try:
            r = subprocess.run([sys.executable, "-c", CHILD, str(b), str(a.replays), str(reuse), str(ls)], env=env,
                               capture_output=True, text=True, timeout=a.timeout)
            rc, tail = r.returncode, (r.stdout + r.stderr).strip().splitlines()[-1:]
        except subprocess.TimeoutExpired:
            rc, tail = "timeout", []
        row = {"queues": q, "branches": b, "reuse_launch_stream": reuse, "launch_on_side": ls, "rc": rc,
               "tail": tail[0][:120] if tail else ""}
        rows.append(row)
        print(json.dumps(row), flush=True)
    bad = [r for r in rows if r["rc"] not in (0,)]
    print(f"{len(bad)} of {len(rows)} cases failed", flush=True)


if __name__ == "__main__":
    main()
