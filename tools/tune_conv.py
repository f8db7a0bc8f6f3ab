#!/usr/bin/env python3
"""Tile autotuner for the implicit-GEMM conv kernels (fwd with BN prologue + stats epilogue, dgrad).

For every conv of a ResNet at a given batch / image size, times every legal tile config
interleaved in one process (median of rounds, random data) and writes the winners to
``dbx_distributed_pytorch_examples_amd/ops/tune_table.json`` (consulted by ops.kernels.pick_tile).
  python tools/tune_conv.py --model resnet50 --batch 1024 --image 224
"""
import argparse
import json
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from dbx_distributed_pytorch_examples_amd.ops import kernels as K  # noqa: E402

TILES = [(128, 128), (128, 64), (64, 64), (256, 128), (128, 256), (256, 64)]
WGRAD_TILES = [(128, 128), (128, 64), (64, 128), (64, 64), (256, 128), (128, 256), (256, 256)]


def convs_of(model_name, image, num_classes=1000):
    from dbx_distributed_pytorch_examples_amd.engine.program import ResNetProgram
    from dbx_distributed_pytorch_examples_amd.models import build_model
    m = build_model(model_name, num_classes=num_classes)
    p = ResNetProgram.__new__(ResNetProgram)
    p.model, p.N, p.H, p.W = m, 1, image, image
    p._build_layers()
    seen = {}
    for cv in p.convs[1:]:
        key = (cv.IC, cv.OC, cv.R, cv.stride, cv.IH)
        seen[key] = seen.get(key, 0) + 1
    return seen


def timeit(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--out", default=os.path.join(ROOT, "dbx_distributed_pytorch_examples_amd", "ops", "tune_table.json"))
    ap.add_argument("--report", default=None)
    ap.add_argument("--verbose", action="store_true", help="print every candidate's median time")
    ap.add_argument("--modes", default="fwd,fwdt,dgrad0,dgrad1,dgrad2,dgrad1b,dgrad2b,wgrad")
    ap.add_argument("--dma", type=int, default=1,
                    help="also time the LDS-DMA operand paths of the fwd / dgrad kernels (tile x path)")
    ap.add_argument("--fast", type=float, default=0.0,
                    help="eight-wave mode: time only the current table entry against the eight-wave kernel "
                         "(csrc/conv_fast.hip, tile dma 4 / 5) on the plain-operand stride-1 fwd0 / dgrad1 / "
                         "dgrad2 convs; an eight-wave tile replaces the entry only when it is this fraction "
                         "faster (e.g. 0.04)")
    ap.add_argument("--wgrad-rounds", default="",
                    help="comma list of split depths (workgroup rounds; 0 = no split) to time for each wgrad with "
                         "its current table tile / operand path; the winner becomes the entry's 4th field")
    a = ap.parse_args()
    dev = "cuda"
    N = a.batch
    table = {}
    if os.path.exists(a.out):
        with open(a.out) as f:
            table = json.load(f)
    lines = ["| C→K | R s | H | count | mode | best tile | ms | TF/s | default tile ms |", "|---|---|---|---|---|---|---|---|---|"]
    for (C, Kc, R, st, H), cnt in convs_of(a.model, a.image).items():
        pad = R // 2
        OH = (H + 2 * pad - R) // st + 1
        x = torch.randn(N, H, H, C, device=dev).bfloat16()
        w = (torch.randn(Kc, R, R, C, device=dev) / math.sqrt(C * R * R)).bfloat16()
        w2 = w.view(Kc, -1)
        wt = w.permute(3, 1, 2, 0).contiguous().view(C, -1)
        y = torch.empty(N, OH, OH, Kc, device=dev, dtype=torch.bfloat16)
        dy = torch.randn(N, OH, OH, Kc, device=dev).bfloat16()
        dx = torch.empty_like(x)
        stats = K.new_stats(Kc, dev)
        sc, sh = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1
        gf = 2.0 * N * OH * OH * Kc * C * R * R / 1e9
        ybn = torch.randn_like(x)
        mref = torch.randn_like(x)
        add = torch.randn_like(x)
        st1 = K.new_stats(C, dev)
        mean, inv = torch.randn(C, device=dev) * 0.1, torch.rand(C, device=dev) + 0.5
        # the BN prologue only exists on inputs that are BN outputs inside a block (<= 512 channels);
        # block inputs (1x1 conv1 / downsample of 1024+ channels) are materialised activations
        psc, psh = (sc, sh) if C <= 512 else (None, None)
        jobs = [("fwd0", N * OH * OH, Kc, C, R, st,
                 lambda t: K.conv_fwd(x, w2, y, R=R, S=R, stride=st, pad=pad, stats=stats, tile=t)),
                ("fwd", N * OH * OH, Kc, C, R, st,
                 lambda t: K.conv_fwd(x, w2, y, R=R, S=R, stride=st, pad=pad, stats=stats, in_scale=psc,
                                      in_shift=psh, tile=t))]
        if R == 1 and st == 1 and Kc < C and K.tail_supported(C, R, R, st, pad):
            # bottleneck conv1 consuming the previous block's output through the tail prologue
            tres, tout = torch.randn_like(x), torch.empty_like(x)
            tbits = torch.empty(x.numel() // 8, device=dev, dtype=torch.uint8)
            jobs.append(("fwdt", N * OH * OH, Kc, C, R, st,
                         lambda t: K.conv_fwd(x, w2, y, R=R, S=R, stride=st, pad=pad, stats=stats, in_scale=sc,
                                              in_shift=sh, tile=t, tail_res=tres, tail_out=tout, tail_bits=tbits)))
        if st > 1 and R == 1:
            # strided 1x1 (downsample): the program runs a dense dgrad onto the subsampled grid
            dxs = torch.empty(N, OH, OH, C, device=dev, dtype=torch.bfloat16)
            jobs.append(("dgrad0", N * OH * OH, C, Kc, 1, 1,
                         lambda t: K.conv_dgrad(dy, wt, dxs, R=1, S=1, stride=1, pad=0, tile=t)))
        else:
            e1 = K.BNBwdEpilogue(K.MASK_OUT, ybn, mean, inv, st1, mbits=K.pack_mask_bits(mref))
            act = torch.empty_like(x)  # the program's MASK_Y dgrads also store the BN output
            e2 = K.BNBwdEpilogue(K.MASK_Y, ybn, mean, inv, st1, scale=sc, shift=sh, act_out=act)
            Md = N * H * H // (st * st)
            jobs.append(("dgrad1", Md, C, Kc, R, st, lambda t: K.conv_dgrad(dy, wt, dx, R=R, S=R, stride=st, pad=pad,
                                                                            tile=t, addsrc=add, epilogue=e1)))
            jobs.append(("dgrad2", Md, C, Kc, R, st, lambda t: K.conv_dgrad(dy, wt, dx, R=R, S=R, stride=st, pad=pad,
                                                                            tile=t, epilogue=e2)))
            if K.tail_supported(Kc, R, R, st, pad):  # 1x1 dgrads with the BN-backward apply prologue
                by, bc, bo = torch.randn_like(dy), torch.randn(3 * Kc, device=dev) * 0.5, torch.empty_like(dy)
                bk = dict(bwd_y=by, bwd_coeff=bc, dy_out=bo)
                jobs.append(("dgrad1b", Md, C, Kc, R, st,
                             lambda t: K.conv_dgrad(dy, wt, dx, R=R, S=R, stride=st, pad=pad, tile=t, addsrc=add,
                                                    epilogue=e1, **bk)))
                jobs.append(("dgrad2b", Md, C, Kc, R, st,
                             lambda t: K.conv_dgrad(dy, wt, dx, R=R, S=R, stride=st, pad=pad, tile=t, epilogue=e2,
                                                    **bk)))
        ws = torch.empty(max(64 * Kc * R * R * C, 16 << 20), device=dev)
        dw = torch.empty(Kc * R * R * C, device=dev)
        # wgrads read stored activations (no BN prologue) since the dgrad-epilogue write-back
        jobs.append(("wgrad", N * OH * OH, Kc, C, R, st,
                     lambda t: K.conv_wgrad(dy, x, dw, ws, R=R, S=R, stride=st, pad=pad, tile=t[:2], dma=t[2],
                                            rounds=t[3] if len(t) > 3 else None)))
        for mode, M, OCm, Kin, Rk, sk, make in jobs:
            if mode not in a.modes.split(","):
                continue
            cur = table.get(K.tune_key(mode, M, OCm, Kin, Rk, sk))
            if a.fast:
                # plain operands, stride 1 (the eight-wave kernel's geometry); dgrad2's MASK_Y epilogue is
                # 128-wide only (conv_fast.hip)
                if mode not in ("fwd0", "dgrad1", "dgrad2") or sk != 1 or OCm % 128:
                    continue
                fb = (128,) if mode == "dgrad2" or OCm % 256 else (128, 256)
                base = tuple(cur) if cur is not None else K.pick_tile(M, OCm, use_table=False)
                cands = [base] + [(256, b, d) for b in fb for d in (4, 5)]
            elif mode == "fwd0":
                continue  # (only in --fast mode: the plain forward is tuned against the eight-wave kernel)
            elif mode == "wgrad" and a.wgrad_rounds:  # split depth for the entry's tile / operand path
                cur = table.get(K.tune_key(mode, M, OCm, Kin, Rk, sk))
                base = tuple(cur[:3]) if cur is not None and len(cur) >= 3 else (
                    128 if Kc % 128 == 0 else 64, 128 if C % 128 == 0 else 64, 2)
                cands = [base + (float(r),) for r in a.wgrad_rounds.split(",")]
            elif mode == "wgrad":  # tile x operand path (LDS-DMA ring depth 3 / 2, 0 = register staged)
                # (256 x 256: LDS-DMA only -- 4 = 32-pixel stages in a 4-slot ring, 2 = 64-pixel stages)
                cands = [t + (d,) for t in WGRAD_TILES if Kc % t[0] == 0 and C % t[1] == 0
                         for d in ((4, 2) if t == (256, 256) else (3, 2, 0))]
            else:  # tile x operand path: prologue convs 0 / 1 (weights by DMA) / 7 (1x1 row tile), plain
                # 0 / 2 / 3 (ring) / 6 (4-slot ring of 32-channel stages)
                pro = mode in ("fwdt", "dgrad1b", "dgrad2b") or (mode == "fwd" and psc is not None)
                dmas = ((0, 1) if pro else (0, 2, 3, 6)) if a.dma else (0,)
                cands = [t + (d,) for t in TILES if OCm % t[1] == 0 for d in dmas]
            res = {t: [] for t in cands}
            for _ in range(a.rounds):
                for t in cands:
                    res[t].append(timeit(lambda t=t: make(t), a.iters))
            med = {t: sorted(v)[len(v) // 2] for t, v in res.items()}
            best = min(med, key=med.get)
            if a.verbose:
                print(f"  {mode} {C}->{Kc} {R}x{R} s{st} @{H}: " + "  ".join(
                    f"{'x'.join(map(str, t))}={v:.3f}" for t, v in sorted(med.items())), flush=True)
            default = (K.pick_tile(M, OCm, use_table=False) + (0,) if mode != "wgrad" else
                       (128 if Kc % 128 == 0 else 64, 128 if C % 128 == 0 else 64, 0))
            if mode == "wgrad" and a.wgrad_rounds:
                default = cands[0][:3] + (2.0,)
            key = K.tune_key(mode, M, OCm, Kin, Rk, sk)
            if a.fast:
                default = cands[0]
                if best != cands[0] and med[best] > (1.0 - a.fast) * med[cands[0]]:
                    best = cands[0]  # not a clear win: keep the entry
                if best == cands[0] and cur is None:
                    continue  # nothing to record
            table[key] = list(best) if (mode == "wgrad" or (len(best) > 2 and best[2])) else list(best[:2])
            lines.append(f"| {C}→{Kc} | {R}x{R} s{st} | {H} | {cnt} | {mode} | {'x'.join(map(str, best))} | {med[best]:.3f} | "
                         f"{gf / med[best]:.0f} | {med.get(default, float('nan')):.3f} |")
            print(lines[-1], flush=True)
    with open(a.out, "w") as f:
        json.dump(table, f, indent=1, sort_keys=True)
    if a.report:
        with open(a.report, "w") as f:
            f.write(f"# conv tile tuning, {a.model} batch {N} image {a.image}\n\n" + "\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
