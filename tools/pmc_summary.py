#!/usr/bin/env python3
"""Summarise per-kernel PMC counters from rocprofv3 ``--pmc`` passes (tools/gpu/pmc_step.sh).

  python tools/pmc_summary.py gpurun_out/pmc_step [--top 40]

Reads every ``*counter_collection.csv`` under the directory (one per pass), joins the passes per
kernel name and prints, per kernel (summed over its dispatches, sorted by device time):

  ms        summed dispatch time of the pass-a run (profiled clocks run a few % low)
  mfma%     SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 1024 SIMDs): matrix-pipe busy
            share per SIMD (GRBM_GUI_ACTIVE is summed over the 8 XCDs; the MFMA busy cycles over all
            1024 SIMDs, 16 per v_mfma_f32_16x16x32_bf16)
  TF/s      SQ_INSTS_MFMA * 16384 FLOP / dispatch time (bf16 16x16x32 MFMAs)
  GHz       effective clock GRBM_GUI_ACTIVE / 8 / time
  valu/mf   SQ_INSTS_VALU / SQ_INSTS_MFMA (a 16x16x32 MFMA leaves ~2 VALU issue slots free)
  wait%     SQ_WAIT_ANY / SQ_WAVE_CYCLES (parked on s_waitcnt / barrier)
  stall%    SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES (issue stalls: pipe busy / dependency)
  lds_cf%   SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  l2hit%    TCC_HIT / (TCC_HIT + TCC_MISS)
  rdTB/s    2 x FETCH_SIZE (KB) / time: gfx950's FETCH_SIZE counts half the bytes of wide
            coalesced reads (MI355X_MICROARCH.md, HBM); Infinity-Cache hits are included
  wrTB/s    WRITE_SIZE (KB) / time
"""
import argparse
import collections
import csv
import glob
import os
import sys


def load(d):
    per = collections.defaultdict(lambda: collections.defaultdict(float))  # kernel -> counter -> sum
    dur = collections.defaultdict(dict)  # kernel -> dispatch -> ns (pass-local)
    calls = collections.defaultdict(set)
    for f in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
        tag = os.path.relpath(f, d).split(os.sep)[0]
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = r.get("Kernel_Name", "?")
                did = r.get("Dispatch_Id", "0")
                per[k][r["Counter_Name"]] += float(r["Counter_Value"])
                calls[k].add((tag, did))
                try:
                    dur[k][(tag, did)] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                except (KeyError, ValueError):
                    pass
    return per, dur, calls


def short(name, n=90):
    name = name.replace("dbx::", "").replace("(dbx::IGemmArgs)", "").replace("(dbx::WgradArgs)", "")
    return name if len(name) <= n else name[:n - 3] + "..."


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    per, dur, calls = load(a.dir)
    if not per:
        print("no counter_collection.csv found", file=sys.stderr)
        return 1
    rows = []
    for k, c in per.items():
        # time from the first pass only (both passes time the same dispatches)
        ds = dur[k]
        tags = sorted({t for t, _ in ds})
        ms = sum(v for (t, _), v in ds.items() if t == tags[0]) / 1e6 if tags else 0.0
        n = len({d for t, d in calls[k] if t == (tags[0] if tags else t)})
        g = c.get("GRBM_GUI_ACTIVE", 0.0)
        simd_cycles = g / 8.0 * 1024  # per-XCD cycles x SIMDs of the whole GPU
        mf = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / simd_cycles if simd_cycles else 0.0
        vpm = c.get("SQ_INSTS_VALU", 0.0) / c["SQ_INSTS_MFMA"] if c.get("SQ_INSTS_MFMA") else float("nan")
        wc = c.get("SQ_WAVE_CYCLES", 0.0)
        wait = c.get("SQ_WAIT_ANY", 0.0) / wc if wc else float("nan")
        stall = c.get("SQ_WAIT_INST_ANY", 0.0) / wc if wc else float("nan")
        lds = c.get("SQ_LDS_BANK_CONFLICT", 0.0) / c["SQ_LDS_IDX_ACTIVE"] if c.get("SQ_LDS_IDX_ACTIVE") else float("nan")
        h, m = c.get("TCC_HIT_sum", 0.0), c.get("TCC_MISS_sum", 0.0)
        l2 = h / (h + m) if h + m else float("nan")
        tfs = c.get("SQ_INSTS_MFMA", 0.0) * 16384 / (ms * 1e-3) / 1e12 if ms else 0.0
        ghz = g / 8.0 / (ms * 1e-3) / 1e9 if ms else 0.0
        rd = 2 * c.get("FETCH_SIZE", float("nan")) * 1024 / (ms * 1e-3) / 1e12 if ms else float("nan")
        wr = c.get("WRITE_SIZE", float("nan")) * 1024 / (ms * 1e-3) / 1e12 if ms else float("nan")
        rows.append((ms, n, mf, tfs, ghz, vpm, wait, stall, lds, l2, rd, wr, k))
    rows.sort(reverse=True)
    tot = sum(r[0] for r in rows)
    print(f"# {len(rows)} kernels, {tot:.2f} ms summed dispatch time (profiled, eager, no wgrad overlap)")
    print(f"{'ms':>8} {'%':>5} {'n':>4} {'mfma%':>6} {'TF/s':>6} {'GHz':>5} {'valu/mf':>7} {'wait%':>6} {'stall%':>6} {'ldscf%':>6} {'l2hit%':>6} {'rdTB/s':>6} {'wrTB/s':>6}  kernel")
    for ms, n, mf, tfs, ghz, vpm, wait, stall, lds, l2, rd, wr, k in rows[:a.top]:
        print(f"{ms:8.3f} {100 * ms / tot:5.1f} {n:4d} {100 * mf:6.1f} {tfs:6.0f} {ghz:5.2f} {vpm:7.2f} {100 * wait:6.1f} {100 * stall:6.1f} "
              f"{100 * lds:6.1f} {100 * l2:6.1f} {rd:6.2f} {wr:6.2f}  {short(k)}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
