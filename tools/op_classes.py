#!/usr/bin/env python3
"""Class totals of a tools/op_breakdown.py report (the VERDICT's kernel classes).

  python tools/op_classes.py op_breakdown.txt

short-K 1x1: 1x1 stride-1 forward / data-gradient GEMMs of depth K <= 512 at 28x28 and below (the
  bottleneck conv3 forwards C -> 4C and conv1 data gradients 4C <- C) plus the fused conv3 backward
  at 28x28; 3x3 @28 / @14 / @7: every stride-1 3x3 fwd / dgrad / wgrad of that map (PF/s = summed
  FLOPs / summed time); per class: calls, ms per step, achieved TF/s.
"""
import re
import sys

LINE = re.compile(r"^(fwd|dgrad|wgrad|dwfused) (\d+)->(\d+) (\dx\d)(?: s(\d))? @(\d+)(.*?)\s+(\d+)\s+([\d.]+)\s+(\d+)\s+([\d.]+)$")


def main(path):
    ops = []
    for ln in open(path):
        m = LINE.match(ln.strip())
        if m:
            kind, a, b, rs, s, hw, rest, calls, ms, tf, tb = m.groups()
            ops.append(dict(kind=kind, a=int(a), b=int(b), rs=rs, s=int(s or 1), hw=int(hw), rest=rest.strip(),
                            calls=int(calls), ms=float(ms), tf=float(tf)))
    classes = {
        "short-K 1x1 (fwd / dgrad K <= 512 at <= 28, dwfused @28)":
            lambda o: (o["kind"] in ("fwd", "dgrad") and o["rs"] == "1x1" and o["s"] == 1 and o["a"] <= 512
                       and o["hw"] <= 28) or (o["kind"] == "dwfused" and o["hw"] == 28),
        "3x3 s1 @28": lambda o: o["rs"] == "3x3" and o["s"] == 1 and o["hw"] == 28,
        "3x3 s1 @14": lambda o: o["rs"] == "3x3" and o["s"] == 1 and o["hw"] == 14,
        "3x3 s1 @7": lambda o: o["rs"] == "3x3" and o["s"] == 1 and o["hw"] == 7,
        "folded (TAIL) dgrads": lambda o: o["kind"] == "dgrad" and "fold" in o["rest"],
    }
    print(f"{'class':60s} {'calls':>5s} {'ms':>7s} {'TF/s':>6s}")
    for name, f in classes.items():
        sel = [o for o in ops if f(o)]
        ms = sum(o["ms"] for o in sel)
        fl = sum(o["tf"] * o["ms"] for o in sel)  # TF/s x ms = GFLOP
        print(f"{name:60s} {sum(o['calls'] for o in sel):5d} {ms:7.3f} {fl / ms if ms else 0:6.0f}")
        for o in sel:
            print(f"    {o['kind']} {o['a']}->{o['b']} {o['rs']} s{o['s']} @{o['hw']} {o['rest']}: "
                  f"{o['calls']} calls {o['ms']:.3f} ms {o['tf']:.0f} TF/s")


if __name__ == "__main__":
    main(sys.argv[1])
