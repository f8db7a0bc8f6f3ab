#!/usr/bin/env python3
"""Per-step timeline of a graph-replayed step from a rocprofv3 kernel trace: for the last steps, the
time each hardware queue is busy, the time both are (overlap), and the step's phases in order --
where the main chain waits on the side stream and what runs alone at the end of the step.

  python tools/step_timeline.py run_kernel_trace.csv|run_results.db [--steps 2] [--tail 12]
A step starts at each augment_u8 (input normalisation) kernel."""
import argparse
import csv
import re


def short(n, w=70):
    n = re.sub(r"\(.*", "", n).replace("void ", "").replace("dbx::", "")
    return n[:w]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--tail", type=int, default=15, help="last kernels listed (0: none)")
    ap.add_argument("--gap-us", type=float, default=20.0)
    ap.add_argument("--top-gaps", type=int, default=12)
    a = ap.parse_args()
    rows = []
    if a.trace.endswith(".db"):  # rocprofv3's default rocpd (SQLite) output
        import sqlite3
        with sqlite3.connect(a.trace) as c:
            rows = [(int(s), int(e), int(q), n) for s, e, q, n in
                    c.execute("select start, end, queue_id, name from kernels")]
    else:
        with open(a.trace) as f:
            for r in csv.DictReader(f):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]), r["Kernel_Name"]))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if "augment_u8" in r[3]]
    for si in range(max(0, len(starts) - 1 - a.steps), len(starts) - 1):
        seg = rows[starts[si]:starts[si + 1]]
        t0, t1 = seg[0][0], rows[starts[si + 1]][0]
        queues = sorted({r[2] for r in seg})
        # busy intervals per queue (union)
        def union(iv):
            iv = sorted(iv)
            out = []
            for s, e in iv:
                if out and s <= out[-1][1]:
                    out[-1][1] = max(out[-1][1], e)
                else:
                    out.append([s, e])
            return out
        busy = {q: union([(r[0], r[1]) for r in seg if r[2] == q]) for q in queues}
        def length(iv):
            return sum(e - s for s, e in iv)
        def inter(x, y):
            i = j = 0
            out = 0
            while i < len(x) and j < len(y):
                s, e = max(x[i][0], y[j][0]), min(x[i][1], y[j][1])
                if s < e:
                    out += e - s
                if x[i][1] < y[j][1]:
                    i += 1
                else:
                    j += 1
            return out
        print(f"step {si}: wall {(t1 - t0) / 1e6:.3f} ms, kernels {len(seg)}")
        for q in queues:
            print(f"  queue {q}: busy {length(busy[q]) / 1e6:.3f} ms, {sum(1 for r in seg if r[2] == q)} kernels")
        if len(queues) == 2:
            ov = inter(busy[queues[0]], busy[queues[1]])
            print(f"  both queues busy {ov / 1e6:.3f} ms")
        # no queue busy at all: dispatch gaps between dependent kernels (by size)
        anyb = union([(r[0], r[1]) for r in seg])
        holes = [anyb[i + 1][0] - anyb[i][1] for i in range(len(anyb) - 1)] + [t1 - anyb[-1][1]]
        hist = {lim: sum(1 for h in holes if h < lim * 1e3) for lim in (2, 5, 20)}
        print(f"  GPU idle (no queue busy): {sum(holes) / 1e6:.3f} ms in {len(holes)} holes "
              f"(< 2 us: {hist[2]}, < 5 us: {hist[5]}, < 20 us: {hist[20]}; mean {sum(holes) / max(1, len(holes)) / 1e3:.2f} us)")
        # idle stretches of each queue inside the step (>= gap_us) and what the other queue ran then
        for q in queues:
            iv = busy[q]
            gaps = [(iv[i][1], iv[i + 1][0]) for i in range(len(iv) - 1) if iv[i + 1][0] - iv[i][1] >= a.gap_us * 1e3]
            tot = sum(e - s for s, e in gaps)
            print(f"  queue {q} idle inside the step: {tot / 1e6:.3f} ms in {len(gaps)} stretches >= {a.gap_us} us")
            for s0, e0 in sorted(gaps, key=lambda g: g[0] - g[1])[:a.top_gaps]:
                other = [r for r in seg if r[2] != q and r[0] < e0 and r[1] > s0]
                names = ", ".join(sorted({short(r[3], 40) for r in other}))[:150]
                print(f"    {(s0 - t0) / 1e6:8.3f} ms +{(e0 - s0) / 1e3:7.1f} us   other queue: {names}")
        print(f"  last {a.tail} kernels (queue, start offset ms, duration us, name):")
        for r in (seg[-a.tail:] if a.tail > 0 else []):
            print(f"    q{r[2]} {(r[0] - t0) / 1e6:8.3f} {(r[1] - r[0]) / 1e3:8.1f}  {short(r[3])}")
    return 0


if __name__ == "__main__":
    main()
