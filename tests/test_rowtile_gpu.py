"""Row-tile kernel (csrc/conv_rowtile.hip, tile code 7): one workgroup per BM-row block over every N
tile, the prologue-transformed A block resident in LDS, the weights streamed through an LDS-DMA ring.

It runs the same MFMA sequence per output tile as the implicit-GEMM kernel (K blocks in order, the
same 16x16x32 fragments), so the conv outputs, the tail / fold write-backs and -- at BM 128, where
its (row block, N tile) partials are the 128 x 128 tiles' -- the BN statistics / moments are
BIT-identical to the four-wave 128 x 128 kernel (test_kernels_gpu.py checks that one against fp32
PyTorch); at BM 64 (K > 256) the statistics are compared to a tolerance and the output to fp32.
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

dev = "cuda"


def K():
    from dbx_distributed_pytorch_examples_amd.ops import kernels
    return kernels


def _stats(st, C):
    return st.view(-1, 2, C).sum(0)


@pytest.mark.parametrize("N,H,IC,OC,tail", [(2, 14, 64, 256, False), (3, 9, 128, 512, False), (2, 14, 256, 1024, False),
                                            (2, 7, 512, 2048, False), (2, 14, 256, 256, True), (2, 7, 512, 512, True),
                                            (5, 13, 192, 384, False)])
def test_rowtile_fwd_matches_implicit_gemm(N, H, IC, OC, tail):
    k = K()
    torch.manual_seed(IC + OC)
    x = torch.randn(N, H, H, IC, device=dev).bfloat16()
    sc, sh = torch.rand(IC, device=dev) + 0.5, torch.randn(IC, device=dev) * 0.1
    w = (torch.randn(OC, IC, device=dev) / math.sqrt(IC)).bfloat16()
    res = torch.randn_like(x) if tail else None
    rsc, rsh = (torch.rand(IC, device=dev) + 0.5, torch.randn(IC, device=dev) * 0.1) if tail else (None, None)

    def run(tile):
        y = torch.empty(N, H, H, OC, device=dev, dtype=torch.bfloat16)
        st = k.new_stats(OC, dev)
        kw = {}
        out = bits = None
        if tail:
            out = torch.full_like(x, float("nan"))
            bits = torch.zeros(x.numel() // 8, device=dev, dtype=torch.uint8)
            kw = dict(tail_res=res, tail_res_scale=rsc, tail_res_shift=rsh, tail_out=out, tail_bits=bits)
        k.conv_fwd(x, w, y, R=1, S=1, stride=1, pad=0, stats=st, in_scale=sc, in_shift=sh, tile=tile, **kw)
        torch.cuda.synchronize()
        return y, _stats(st, OC), out, bits

    y0, s0, o0, b0 = run((128, 128, 0))
    y1, s1, o1, b1 = run((128, 128, 7))
    assert torch.equal(y0, y1)
    if tail:
        assert torch.equal(o0, o1) and torch.equal(b0, b1)
    if IC <= 256:
        assert torch.equal(s0, s1)
    else:
        assert torch.allclose(s0, s1, rtol=1e-5, atol=1e-2)
    # and against fp32 torch
    a = x.float() * sc + sh
    if tail:
        a = a + res.float() * rsc + rsh
    a = torch.relu(a).bfloat16().float()
    ref = (a.view(-1, IC) @ w.float().t()).view(N, H, H, OC)
    assert (y1.float() - ref).abs().max() / ref.abs().max() < 1e-2


@pytest.mark.parametrize("Kc,Cc", [(64, 256), (128, 512), (256, 1024), (512, 2048), (128, 384)])
@pytest.mark.parametrize("variant", ["epi1_acc", "epi2", "plain", "acc"])
def test_rowtile_fold_dgrad_matches_implicit_gemm(Kc, Cc, variant):
    k = K()
    N, H = 2, 13
    torch.manual_seed(Kc * 3 + Cc)
    g = torch.randn(N, H, H, Kc, device=dev).bfloat16()
    y = torch.randn_like(g)
    coeff = torch.randn(3 * Kc, device=dev) * 0.5
    wt = (torch.randn(Cc, Kc, device=dev) / math.sqrt(Kc)).bfloat16()
    ybn = torch.randn(N, H, H, Cc, device=dev).bfloat16()
    ybn2 = torch.randn_like(ybn)
    mean, inv = torch.randn(Cc, device=dev) * 0.1, torch.rand(Cc, device=dev) + 0.5
    mean2, inv2 = torch.randn(Cc, device=dev) * 0.1, torch.rand(Cc, device=dev) + 0.5
    sc, sh = torch.rand(Cc, device=dev) + 0.5, torch.randn(Cc, device=dev) * 0.1
    add = torch.randn_like(ybn)
    mbits = k.pack_mask_bits(torch.randn_like(ybn))

    def run(tile):
        s1, s2 = k.new_stats(Cc, dev), k.new_stats(Cc, dev)
        dx = torch.empty(N, H, H, Cc, device=dev, dtype=torch.bfloat16)
        dy_out = torch.full_like(g, float("nan"))
        act = torch.full_like(ybn, float("nan"))
        kw = dict(bwd_y=y, bwd_coeff=coeff, dy_out=dy_out, tile=tile)
        if variant == "epi2":
            kw["epilogue"] = k.BNBwdEpilogue(k.MASK_Y, ybn, mean, inv, s1, scale=sc, shift=sh, act_out=act)
        elif variant == "epi1_acc":
            kw.update(epilogue=k.BNBwdEpilogue(k.MASK_OUT, ybn, mean, inv, s1, mbits=mbits, ybn2=ybn2, mean2=mean2,
                                               inv2=inv2, stats2=s2), addsrc=add)
        elif variant == "acc":
            kw["addsrc"] = add
        k.conv_dgrad(g, wt, dx, R=1, S=1, stride=1, pad=0, **kw)
        torch.cuda.synchronize()
        return dx, dy_out, act, _stats(s1, Cc), _stats(s2, Cc)

    r0, r1 = run((128, 128, 0)), run((128, 128, 7))
    assert torch.equal(r0[0], r1[0]) and torch.equal(r0[1], r1[1])
    if variant == "epi2":
        assert torch.equal(r0[2], r1[2])
    if variant in ("epi2", "epi1_acc"):
        for a, b in ((r0[3], r1[3]), (r0[4], r1[4])):
            if Kc <= 256:
                assert torch.equal(a, b)
            else:
                assert torch.allclose(a, b, rtol=1e-5, atol=1e-2)
    # the applied operand against fp32
    dyr = (g.float() * coeff[:Kc] + coeff[2 * Kc:] + y.float() * coeff[Kc:2 * Kc]).bfloat16()
    assert (r1[1].float() - dyr.float()).abs().max() <= 0.02 * dyr.float().abs().max()
    if variant == "plain":
        ref = (dyr.float().view(-1, Kc) @ wt.float().t()).view(N, H, H, Cc)
        assert (r1[0].float() - ref).abs().max() / ref.abs().max() < 1e-2


def test_rowtile_rejects_unsupported():
    k = K()
    x = torch.randn(2, 8, 8, 1024, device=dev).bfloat16()
    w = torch.randn(256, 1024, device=dev).bfloat16()
    y = torch.empty(2, 8, 8, 256, device=dev, dtype=torch.bfloat16)
    st = k.new_stats(256, dev)
    sc, sh = torch.ones(1024, device=dev), torch.zeros(1024, device=dev)
    with pytest.raises(RuntimeError):  # K = 1024 > the resident A image (512 at BM 64)
        k.conv_fwd(x, w, y, R=1, S=1, stride=1, pad=0, stats=st, in_scale=sc, in_shift=sh, tile=(128, 128, 7))
