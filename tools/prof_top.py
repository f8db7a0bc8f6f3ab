#!/usr/bin/env python3
"""Summarise a rocprofv3 ``--stats`` kernel_stats.csv: the top kernels by total time, per step.

  python tools/prof_top.py <kernel_stats.csv> [steps] [top]
``steps``: profiled steps (the per-step column divides by it)."""
import csv
import sys


def main():
    path = sys.argv[1]
    steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    rows = list(csv.DictReader(open(path)))
    tot_key = next(k for k in rows[0] if "Total" in k and "Duration" in k)
    calls_key = next(k for k in rows[0] if k.lower().startswith("calls"))
    rows.sort(key=lambda r: -float(r[tot_key]))
    total = sum(float(r[tot_key]) for r in rows) / 1e6
    print(f"# {path}: {len(rows)} kernels, {total:.2f} ms total, {total / steps:.3f} ms per step ({steps:g} steps)")
    print(f"{'ms/step':>9} {'%':>6} {'calls/step':>10} {'avg us':>8}  kernel")
    for r in rows[:top]:
        t = float(r[tot_key]) / 1e6
        c = float(r[calls_key])
        name = r["Name"] if "Name" in r else r.get("KernelName", "?")
        print(f"{t / steps:9.3f} {100 * t / total:6.1f} {c / steps:10.1f} {1000 * t / c:8.1f}  {name[:150]}")


if __name__ == "__main__":
    main()
