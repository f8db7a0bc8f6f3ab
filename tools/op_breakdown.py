#!/usr/bin/env python3
"""Per-op device time of one native ResNet-50 training step, with a roofline column per op.

Every kernel wrapper the program calls (ops/kernels.py) is wrapped with a hipEvent pair, the
step runs eagerly with the wgrad side stream disabled (so op times do not overlap), and each op
gets FLOP and minimum-HBM-byte estimates -> achieved TF/s and TB/s. Output: the categories
(conv fwd / dgrad / wgrad / BN passes / rest) and the top ops, sorted by time.

  BATCH=1024 python tools/op_breakdown.py [--steps 3] [--top 40]
  ARCH=resnet18 SIZE=32 CLASSES=10 BATCH=256 python tools/op_breakdown.py   (the CIFAR preset)
"""
import argparse
import collections
import os
import sys

os.environ["DBX_ENGINE"] = ",".join(x for x in (os.environ.get("DBX_ENGINE", ""), "overlap_wgrad=0") if x)
import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dbx_distributed_pytorch_examples_amd.engine.native_trainer import NativeTrainer, OptimConfig  # noqa: E402
from dbx_distributed_pytorch_examples_amd.models import build_model  # noqa: E402
from dbx_distributed_pytorch_examples_amd.ops import kernels as K  # noqa: E402

RECS = []


def _b(t):
    return 0 if t is None else t.numel() * t.element_size()


def est(name, args, kw):
    """(label, flops, bytes) of one call."""
    if name == "conv_fwd":
        x, w, out = args[:3]
        N, IH, IW, IC = x.shape
        OC = w.shape[0]
        fl = 2 * out.numel() * w.shape[1]
        by = _b(x) + _b(w) + _b(out) + _b(kw.get("tail_res")) + _b(kw.get("tail_out")) + _b(kw.get("tail_bits"))
        tag = " tail" if kw.get("tail_res") is not None else (" pro" if kw.get("in_scale") is not None else "")
        return f"fwd {IC}->{OC} {kw['R']}x{kw['S']} s{kw['stride']} @{IH}{tag}", fl, by
    if name == "conv_dgrad":
        dy, wt, dx = args[:3]
        N, P, Q, Kc = dy.shape
        fl = 2 * dy.numel() * wt.shape[0] * kw["R"] * kw["S"]
        epi = kw.get("epilogue")
        by = _b(dy) + _b(wt) + _b(dx) + _b(kw.get("addsrc")) + _b(kw.get("bwd_y")) + _b(kw.get("dy_out"))
        if kw.get("accumulate") and kw.get("addsrc") is None:
            by += _b(dx)  # dx += result
        tag = " fold" if kw.get("bwd_y") is not None else ""
        if epi is not None:
            by += _b(epi.ybn) + _b(epi.ybn2) + _b(epi.mbits)
            by += _b(epi.act_out)
            tag += f" epi{epi.mode}"
        return f"dgrad {Kc}->{dx.shape[3]} {kw['R']}x{kw['S']} s{kw['stride']} @{dx.shape[1]}{tag}", fl, by
    if name == "conv_wgrad":
        dy, x, dw = args[:3]
        N, OH, OW, OC = dy.shape
        fl = 2 * dy.numel() * dw.shape[1] if not kw.get("stem") else 2 * dy.numel() * 147
        return f"wgrad {x.shape[3]}->{OC} {kw['R']}x{kw['S']} s{kw['stride']} @{x.shape[1]}", fl, _b(dy) + _b(x) + _b(dw)
    if name == "conv_dwfused":
        g, y3, _, wt, y2 = args[:5]
        da, dw = args[10], args[11]
        fl = 2 * 2 * g.numel() * y2.shape[-1]  # data + weight gradient GEMMs
        return (f"dwfused {g.shape[3]}->{y2.shape[3]} 1x1 @{g.shape[1]}", fl,
                _b(g) + _b(y3) + _b(y2) + _b(da) + _b(wt))
    if name == "stem_bwd_fused":
        dpool, arg, y = args[:3]
        x4 = args[6]
        return "stem bwd fused", 2 * y.numel() * 256, _b(dpool) + _b(arg) + _b(y) + _b(x4)
    if name == "conv_stem_fwd":
        x4, w, out = args[:3]
        return "stem fwd", 2 * out.numel() * 147, _b(x4) + _b(out)
    if name == "bn_apply":
        y, out = args[0], args[3]
        return f"bn_apply {tuple(y.shape[1:])}", 0, _b(y) + _b(out) + _b(kw.get("res")) + _b(kw.get("mbits"))
    if name == "bn_bwd_apply":
        dout, y, dy = args[0], args[1], args[3]
        return f"bn_bwd_apply {tuple(y.shape[1:])}", 0, _b(dout) + _b(y) + _b(dy) + _b(kw.get("gout")) + _b(kw.get("mref"))
    if name == "bn_bwd_reduce":
        dout, y = args[0], args[1]
        return f"bn_bwd_reduce {tuple(y.shape[1:])}", 0, _b(dout) + _b(y) + _b(kw.get("mref"))
    t = args[0] if args and isinstance(args[0], torch.Tensor) else None
    return name, 0, _b(t)


_DEPTH = [0]


def wrap(name):
    fn = getattr(K, name)

    def w(*args, **kw):
        if _DEPTH[0]:  # a wrapper calling itself (the eight-wave batch split): timed by the outer call
            return fn(*args, **kw)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        _DEPTH[0] += 1
        try:
            r = fn(*args, **kw)
        finally:
            _DEPTH[0] -= 1
        e.record()
        RECS.append((name, est(name, args, kw), s, e))
        return r
    setattr(K, name, w)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--top", type=int, default=45)
    a = ap.parse_args()
    B = int(os.environ.get("BATCH", 1024))
    arch = os.environ.get("ARCH", "resnet50")
    hw = int(os.environ.get("SIZE", 224))
    ncls = int(os.environ.get("CLASSES", 1000))
    tr = NativeTrainer(build_model(arch, num_classes=ncls), B, (hw, hw), torch.device("cuda"), optim=OptimConfig(),
                       use_graphs=False)
    tr.prog.img_u8.copy_(torch.randint(0, 256, tr.prog.img_u8.shape, dtype=torch.uint8))
    tr.prog.labels.copy_(torch.randint(0, ncls, (B,)))
    for _ in range(2):
        tr.step()
    torch.cuda.synchronize()
    for n in ["conv_fwd", "conv_dgrad", "conv_wgrad", "conv_dwfused", "stem_bwd_fused", "conv_stem_fwd", "bn_apply", "bn_bwd_apply", "bn_bwd_reduce",
              "bn_bwd_coeff", "bn_finalize", "maxpool_fwd", "maxpool_bwd", "avgpool_fwd", "avgpool_bwd",
              "softmax_ce", "sgd_step", "weight_prep", "augment_u8", "pool_bn_bwd_reduce", "pool_bn_bwd_apply", "bn_bwd_apply2"]:
        wrap(n)
    s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s0.record()
    for _ in range(a.steps):
        tr.step()
    s1.record()
    torch.cuda.synchronize()
    wall = s0.elapsed_time(s1) / a.steps
    agg = collections.OrderedDict()
    for name, (label, fl, by), s, e in RECS:
        ms = s.elapsed_time(e)
        r = agg.setdefault(label, [0.0, 0, 0, 0, name])
        r[0] += ms / a.steps
        r[1] += fl / a.steps
        r[2] += by / a.steps
        r[3] += 1
    cat = collections.Counter()
    for label, (ms, fl, by, n, name) in agg.items():
        cat[name] += ms
    tot = sum(cat.values())
    print(f"batch {B}: wall {wall:.2f} ms/step (eager, no wgrad overlap), wrapped ops {tot:.2f} ms")
    for k, v in cat.most_common():
        print(f"  {k:16s} {v:8.3f} ms  {100 * v / wall:5.1f}%")
    print(f"\n{'op':44s} {'calls':>5s} {'ms':>7s} {'TF/s':>6s} {'TB/s':>5s}")
    for label, (ms, fl, by, n, name) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:a.top]:
        tf = fl / (ms * 1e-3) / 1e12 if ms > 0 else 0
        tb = by / (ms * 1e-3) / 1e12 if ms > 0 else 0
        print(f"{label:44s} {n // a.steps:5d} {ms:7.3f} {tf:6.0f} {tb:5.2f}")


if __name__ == "__main__":
    main()
