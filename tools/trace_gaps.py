#!/usr/bin/env python3
"""Timeline of a rocprofv3 ``--kernel-trace`` run: busy time vs wall time per step and the largest
idle gaps (with the kernels on either side), to find where a step loses time between kernels --
graph-segment boundaries, stream joins, host waits.

  python tools/trace_gaps.py gpurun_out/trace_seg/run_kernel_trace.csv [--last 3] [--top 15]

Steps are delimited by the optimizer kernel (``sgd_kernel`` / ``adam_kernel`` by default); the
last ``--last`` steps are analysed (the earlier ones are warm-up / capture).
"""
import argparse
import csv
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last", type=int, default=3)
    ap.add_argument("--top", type=int, default=15)
    ap.add_argument("--step-marker", default="sgd_kernel,adam_kernel")
    a = ap.parse_args()
    ks, qs = [], {}
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            ks.append((s, e, r["Kernel_Name"]))
            q = r.get("Queue_Id") or r.get("Stream_Id") or "?"
            qs.setdefault(q, []).append((s, e, r["Kernel_Name"]))
    ks.sort()
    markers = tuple(m.strip() for m in a.step_marker.split(","))
    ends = [e for s, e, n in ks if any(m in n for m in markers)]
    if len(ends) < a.last + 1:
        print(f"only {len(ends)} step markers found", file=sys.stderr)
        return 1
    t0, t1 = ends[-a.last - 1], ends[-1]
    win = [(s, e, n) for s, e, n in ks if s >= t0 and e <= t1]
    busy, cur_s, cur_e = 0, None, None
    gaps = []
    prev_name = "(step start)"
    for s, e, n in win:
        if cur_e is None:
            if s > t0:
                gaps.append((s - t0, prev_name, n))
            cur_s, cur_e = s, e
        elif s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, prev_name, n))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        prev_name = n
    if cur_e is not None:
        busy += cur_e - cur_s
    wall = t1 - t0
    sumk = sum(e - s for s, e, _ in win)
    print(f"{a.last} steps: wall {wall / 1e6 / a.last:.3f} ms/step, GPU busy (union) {busy / 1e6 / a.last:.3f} ms/step "
          f"({100 * busy / wall:.1f} %), kernel time summed {sumk / 1e6 / a.last:.3f} ms/step "
          f"(overlap {100 * (sumk - busy) / max(1, busy):.1f} %), {len(win) // a.last} kernels/step")
    # per hardware queue: busy time inside the window (a queue busy ~100 % is the critical path;
    # kernels of the other queues then only matter through the CUs they take from it)
    for q, lst in sorted(qs.items(), key=lambda kv: -len(kv[1])):
        w = sorted((s, e) for s, e, _ in lst if s >= t0 and e <= t1)
        if not w:
            continue
        b, cs, ce = 0, w[0][0], w[0][1]
        for s, e in w[1:]:
            if s > ce:
                b += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        b += ce - cs
        top = {}
        for s, e, n in lst:
            if s >= t0 and e <= t1:
                k = n.split("(")[0][:60]
                top[k] = top.get(k, 0) + e - s
        tops = ", ".join(f"{k} {v / 1e6 / a.last:.2f}" for k, v in sorted(top.items(), key=lambda kv: -kv[1])[:3])
        print(f"queue {q}: {len(w) // a.last} kernels/step, busy {b / 1e6 / a.last:.3f} ms/step "
              f"({100 * b / wall:.1f} % of wall); top: {tops}")
    idle = sum(g for g, _, _ in gaps)
    print(f"idle {idle / 1e6 / a.last:.3f} ms/step in {len(gaps) // a.last} gaps/step; largest:")
    short = lambda n: (n[:70] + "...") if len(n) > 73 else n  # noqa: E731
    for g, p, n in sorted(gaps, reverse=True)[:a.top]:
        print(f"  {g / 1e3:8.1f} us  after {short(p)}\n              before {short(n)}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
