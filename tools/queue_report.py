#!/usr/bin/env python3
"""Per-queue kernel classes of the last replayed steps of a rocprofv3 kernel trace: which hardware
queue the comm branch (scale kernels of comm_loopback / RCCL kernels), the weight-gradient side
stream and the main chain land on, and how often a comm kernel ran on the same queue as a weight
gradient.   python tools/queue_report.py run_kernel_trace.csv|run_results.db [--steps 2]"""
import argparse
import collections
import csv


def kind(name: str) -> str:
    if "nccl" in name.lower() or "rccl" in name.lower() or "MulFunctor" in name or "dar_kernel" in name:
        return "comm"
    if "wgrad" in name:
        return "wgrad"
    return "main"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=2)
    a = ap.parse_args()
    if a.trace.endswith(".db"):
        import sqlite3
        with sqlite3.connect(a.trace) as c:
            rows = [(int(s), int(e), int(q), n) for s, e, q, n in c.execute("select start, end, queue_id, name from kernels")]
    else:
        with open(a.trace) as f:
            rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]), r["Kernel_Name"])
                    for r in csv.DictReader(f)]
    rows.sort()
    starts = [i for i, r in enumerate(rows) if "augment_u8" in r[3]]
    if len(starts) < 2:
        print("no complete step in the trace")
        return 1
    seg = rows[starts[max(0, len(starts) - 1 - a.steps)]:starts[-1]]
    cnt = collections.Counter((r[2], kind(r[3])) for r in seg)
    queues = sorted({q for q, _ in cnt})
    print(f"{len(seg)} kernels in the last {a.steps} steps")
    for q in queues:
        print(f"  queue {q}: " + ", ".join(f"{k} {cnt[(q, k)]}" for k in ("main", "wgrad", "comm") if cnt[(q, k)]))
    comm_q = {q for q in queues if cnt[(q, "comm")]}
    wg_q = {q for q in queues if cnt[(q, "wgrad")]}
    shared = comm_q & wg_q
    print(f"comm queues {sorted(comm_q)}, weight-gradient queues {sorted(wg_q)}; shared: {sorted(shared) or 'none'}")
    # a comm kernel that started while a weight gradient on its queue was still running = queued behind it
    behind = 0
    for s, e, q, n in seg:
        if kind(n) == "comm" and any(r[2] == q and kind(r[3]) == "wgrad" and r[0] < s < r[1] + 2000 for r in seg):
            behind += 1
    print(f"comm kernels started within 2 us of a weight gradient's end on the same queue: {behind}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
