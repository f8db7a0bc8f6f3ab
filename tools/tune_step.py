#!/usr/bin/env python3
"""Step-level tile tuner: picks each conv shape's tile / operand path / split depth by the time of the
WHOLE graph-replayed training step, not of the kernel alone.

``tools/tune_conv.py`` times one kernel at a time on an idle GPU; in the step a main-chain kernel shares
the CUs with the side stream's weight gradients (and the small steps are launch / latency bound), so
a tile that wins alone can lose in the step (round 5: tuning the small-map shapes in isolation made the
TinyImageNet step slower, profiles/r5_tune_small/). Here every candidate is installed in the tune
table, the step graph is re-captured and timed by replay, and a change is kept only when the step gets
faster by more than the noise threshold, confirmed by a second interleaved measurement (greedy
coordinate descent over the shapes the step looks up, largest first, within a time budget).

  python tools/tune_step.py --preset resnet50_tiny_imagenet --budget-s 420 --out gpurun_out/tune_tiny.json

Candidates per shape: the menu of values the table already uses for that kernel mode (the winners of
the isolated tuner across all shapes), filtered to the shape's channel count. Each candidate first runs
one eager step (the launchers reject an illegal tile on the host before anything is captured).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


class Recorder(dict):
    """The tune table, recording every key the step looks up."""

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.seen = []

    def get(self, key, default=None):
        if key not in self.seen:
            self.seen.append(key)
        return super().get(key, default)


def parse_key(k):
    mode, m, n, kk, r, s = k.split(":")
    return mode, int(m[1:]), int(n[1:]), int(kk[1:]), int(r[1:]), int(s[1:])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="resnet50_tiny_imagenet")
    ap.add_argument("--budget-s", type=float, default=420.0)
    ap.add_argument("--steps", type=int, default=0, help="replays per measurement (0: ~0.25 s worth)")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--thresh", type=float, default=0.003, help="relative gain a change must show (twice)")
    ap.add_argument("--max-keys", type=int, default=0)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()

    import bench
    from dbx_distributed_pytorch_examples_amd.ops import kernels as K
    from dbx_distributed_pytorch_examples_amd.parallel import dist as ddist
    from dbx_distributed_pytorch_examples_amd.train.bench_steps import build_step

    # lr 0: thousands of replays on random labels must not drift the weights (timing is the same)
    args = bench.parse_args(([] if a.preset == "headline" else ["--preset", a.preset]) + ["--lr", "0"])
    info = ddist.init_distributed()
    table = Recorder(K._tune_table())
    K._TUNE = table
    step, _ = build_step(args, info)
    tr = step.trainer
    for _ in range(4):  # two eager warm-up steps, the capture, one replay
        step()
    torch.cuda.synchronize()
    keys = [k for k in table.seen if k.count(":") == 5]
    menu = {}
    for k, v in table.items():
        menu.setdefault(k.split(":")[0], set()).add(tuple(v))

    def grads_with(entry, k):
        """One eager step's flat gradient with ``entry`` installed for key ``k`` (None: no entry), from
        the same master weights."""
        if entry is None:
            dict.pop(table, k, None)
        else:
            table[k] = tuple(entry)
        saved = tr.prog.master.clone()
        tr._run_phases_eager()
        torch.cuda.synchronize()
        g = tr.prog.grad.clone()
        tr.prog.master.copy_(saved)
        return g

    def numerics_ok(k, prev, c):
        g0 = grads_with(prev, k)
        g1 = grads_with(c, k)
        rel = ((g1 - g0).norm() / g0.norm().clamp_min(1e-30)).item()
        return rel < 2e-2 and torch.isfinite(g1).all().item(), rel

    def recapture():
        tr.graphs = []
        step()  # capture (+ replay)
        torch.cuda.synchronize()

    def measure(n):
        ts = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(n):
                step()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) / n)
        return min(ts)

    t_probe = measure(5)
    n = a.steps or max(5, int(250.0 / max(t_probe, 0.1)))
    best = measure(n)
    print(f"[tune_step] {a.preset}: {len(keys)} table lookups, baseline {best:.4f} ms/step ({n} replays x {a.reps})",
          flush=True)

    def cost(k):
        mode, M, N, KK, R, s = parse_key(k)
        return M * N * KK * R * R
    order = sorted(keys, key=cost, reverse=True)
    if a.max_keys:
        order = order[:a.max_keys]
    t0 = time.time()
    changes, trials = [], 0
    for k in order:
        mode, M, N, KK, R, s = parse_key(k)
        cur = table.get(k)
        cands = sorted(c for c in menu.get(mode, ()) if N % c[1] == 0 and (cur is None or tuple(cur) != c))
        for c in cands:
            if time.time() - t0 > a.budget_s:
                break
            trials += 1
            prev = dict.get(table, k)
            table[k] = tuple(c)
            try:
                tr._run_phases_eager()  # host-side legality checks before any capture
                torch.cuda.synchronize()
                recapture()
                t = measure(n)
            except Exception as e:  # noqa: BLE001 - an illegal tile for this shape: skip it
                tr.prog.drop_pending()
                torch.cuda.synchronize()
                print(f"  {k} {c}: rejected ({type(e).__name__}: {str(e)[:80]})", flush=True)
                t = None
            keep = False
            if t is not None:
                print(f"  {k} {c}: {t:.4f} ms/step (best {best:.4f}; {time.time() - t0:.0f} s)", flush=True)
            if t is not None and t < best * (1 - a.thresh):
                # confirm: the incumbent again, then the candidate again
                if prev is None:
                    dict.pop(table, k, None)
                else:
                    table[k] = prev
                recapture()
                t_inc = measure(n)
                table[k] = tuple(c)
                recapture()
                t2 = measure(n)
                keep = t2 < t_inc * (1 - a.thresh)
                if keep:
                    ok, rel = numerics_ok(k, prev, c)  # same gradient (summation order aside) as before
                    table[k] = tuple(c)
                    recapture()
                    if not ok:
                        print(f"  {k} {c}: faster but the gradient differs (rel {rel:.2e}): rejected", flush=True)
                        keep = False
                if keep:
                    print(f"  {k}: {prev} -> {c}  {t_inc:.4f} -> {t2:.4f} ms/step", flush=True)
                    changes.append({"key": k, "old": prev, "new": list(c), "ms_old": t_inc, "ms_new": t2})
                    best = t2
            if not keep:
                if prev is None:
                    dict.pop(table, k, None)
                else:
                    table[k] = prev
        else:
            continue
        break  # budget spent
    recapture()
    final = measure(n)
    out = {k: list(v) for k, v in sorted(dict.items(table))}
    with open(a.out, "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)
    print(json.dumps({"preset": a.preset, "trials": trials, "changes": len(changes), "final_ms": round(final, 4),
                      "elapsed_s": round(time.time() - t0, 1), "accepted": changes}), flush=True)


if __name__ == "__main__":
    main()
