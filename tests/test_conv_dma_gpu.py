"""LDS-DMA operand paths of the implicit-GEMM conv kernels (csrc/conv_igemm_kernel.h, DMA 1/2/3).

The DMA paths move the same bytes into the same (swizzled) LDS positions as the register-staged
path and run the same MFMA sequence, so every output -- conv result, BN statistics, BN-backward
moments, the tail / fold write-backs -- must be BIT-identical to the register path (dma=0), which
test_kernels_gpu.py checks against fp32 PyTorch references.
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

dev = "cuda"
TILES = [(128, 128), (128, 64), (64, 64), (256, 128), (128, 256), (256, 64)]


def K():
    from dbx_distributed_pytorch_examples_amd.ops import kernels
    return kernels


@pytest.fixture(autouse=True)
def _no_splitk(engine):
    """The register path splits the K loop of few-tile launches (splitk_wgs) and the ring paths never
    do: compare the operand paths on unsplit launches (split-K has its own tests, test_splitk_gpu.py)."""
    engine(splitk_wgs=0)


def _same(outs0, outs1, what):
    for a, b in zip(outs0, outs1):
        assert torch.equal(a, b), what


@pytest.mark.parametrize("case", [
    # N, H, W, IC, OC, R, stride, pad
    (2, 14, 14, 64, 64, 3, 1, 1),
    (2, 14, 14, 128, 256, 1, 1, 0),
    (2, 14, 14, 256, 512, 1, 2, 0),
    (3, 7, 7, 512, 512, 3, 1, 1),
    (4, 9, 9, 64, 128, 3, 2, 1),
    (5, 13, 11, 192, 128, 3, 1, 1),  # M not a multiple of any tile; 3 channel blocks per tap
])
@pytest.mark.parametrize("prologue", [False, True])
def test_fwd_dma_bit_exact(case, prologue):
    k = K()
    N, H, W, IC, OC, R, st, pad = case
    torch.manual_seed(3)
    x = torch.randn(N, H, W, IC, device=dev).bfloat16()
    w = (torch.randn(OC, R * R * IC, device=dev) / math.sqrt(IC * R * R)).bfloat16()
    OH, OW = k.conv_out_hw(H, W, R, R, st, pad)
    sc = sh = None
    if prologue:
        sc, sh = torch.rand(IC, device=dev) + 0.5, torch.randn(IC, device=dev) * 0.1
    dmas = (1,) if prologue else (2, 3, 6)  # 6: 4-slot ring of 32-channel stages

    def run(tile, dma):
        y = torch.full((N, OH, OW, OC), float("nan"), device=dev, dtype=torch.bfloat16)
        s = k.new_stats(OC, dev)
        k.conv_fwd(x, w, y, R=R, S=R, stride=st, pad=pad, stats=s, in_scale=sc, in_shift=sh, tile=(*tile, dma))
        return y, s

    for tile in TILES:
        if OC % tile[1]:
            continue
        base = run(tile, 0)
        assert not torch.isnan(base[0].float()).any()
        for dma in dmas:
            _same(base, run(tile, dma), (tile, dma))


@pytest.mark.parametrize("case", [
    (2, 14, 14, 64, 64, 3, 1, 1),
    (2, 14, 14, 64, 256, 1, 1, 0),
    (2, 14, 14, 128, 128, 3, 2, 1),
    (3, 7, 7, 512, 512, 3, 1, 1),
    (4, 9, 9, 64, 128, 3, 2, 1),
])
@pytest.mark.parametrize("variant", ["plain", "acc", "epi1_add", "epi2"])
def test_dgrad_dma_bit_exact(case, variant):
    k = K()
    N, H, W, IC, OC, R, st, pad = case
    torch.manual_seed(4)
    OH, OW = k.conv_out_hw(H, W, R, R, st, pad)
    w = (torch.randn(OC, R, R, IC, device=dev) / math.sqrt(IC * R * R)).bfloat16()
    wt = w.permute(3, 1, 2, 0).contiguous().view(IC, -1)
    dy = torch.randn(N, OH, OW, OC, device=dev).bfloat16()
    base_dx = torch.randn(N, H, W, IC, device=dev).bfloat16()
    add = torch.randn(N, H, W, IC, device=dev).bfloat16()
    ybn, ybn2 = torch.randn_like(base_dx), torch.randn_like(base_dx)
    mbits = k.pack_mask_bits(torch.randn_like(base_dx))
    mean, inv = torch.randn(IC, device=dev) * 0.1, torch.rand(IC, device=dev) + 0.5
    sc, sh = torch.rand(IC, device=dev) + 0.5, torch.randn(IC, device=dev) * 0.1

    def run(tile, dma):
        dx = base_dx.clone()
        s1, s2 = k.new_stats(IC, dev), k.new_stats(IC, dev)
        act = torch.full_like(base_dx, float("nan"))
        kw = {}
        if variant == "acc":
            kw = dict(accumulate=True)
        elif variant == "epi1_add":
            kw = dict(addsrc=add, epilogue=k.BNBwdEpilogue(k.MASK_OUT, ybn, mean, inv, s1, mbits=mbits, ybn2=ybn2,
                                                             mean2=mean, inv2=inv, stats2=s2))
        elif variant == "epi2":
            kw = dict(epilogue=k.BNBwdEpilogue(k.MASK_Y, ybn, mean, inv, s1, scale=sc, shift=sh, act_out=act))
        k.conv_dgrad(dy, wt, dx, R=R, S=R, stride=st, pad=pad, tile=(*tile, dma), **kw)
        return dx, s1, s2, torch.nan_to_num(act)

    for tile in TILES:
        if IC % tile[1]:
            continue
        if variant == "epi1_add" and st > 1:
            continue  # (a full-resolution addend with a strided dgrad is not a ResNet pattern)
        base = run(tile, 0)
        for dma in (2, 3, 6):
            _same(base, run(tile, dma), (tile, dma, variant))


@pytest.mark.parametrize("tile", TILES)
def test_fwd_tail_dma_bit_exact(tile):
    k = K()
    N, H, W, IC, OC = 2, 14, 14, 256, 128
    if OC % tile[1]:
        pytest.skip("tile wider than OC")
    torch.manual_seed(5)
    x = torch.randn(N, H, W, IC, device=dev).bfloat16()
    res = torch.randn_like(x)
    sc, sh = torch.rand(IC, device=dev) + 0.5, torch.randn(IC, device=dev) * 0.1
    rsc, rsh = torch.rand(IC, device=dev) + 0.5, torch.randn(IC, device=dev) * 0.1
    w = (torch.randn(OC, IC, device=dev) / math.sqrt(IC)).bfloat16()

    def run(dma, ds):
        out = torch.full_like(x, float("nan"))
        bits = torch.zeros(x.numel() // 8, device=dev, dtype=torch.uint8)
        y, s = torch.empty(N, H, W, OC, device=dev, dtype=torch.bfloat16), k.new_stats(OC, dev)
        k.conv_fwd(x, w, y, R=1, S=1, stride=1, pad=0, stats=s, in_scale=sc, in_shift=sh, tile=(*tile, dma),
                   tail_res=res, tail_res_scale=rsc if ds else None, tail_res_shift=rsh if ds else None,
                   tail_out=out, tail_bits=bits)
        return y, s, out, bits

    for ds in (False, True):
        _same(run(0, ds), run(1, ds), (tile, ds))


@pytest.mark.parametrize("tile", TILES)
@pytest.mark.parametrize("variant", ["epi2", "epi1_acc", "plain"])
def test_dgrad_fold_dma_bit_exact(tile, variant):
    k = K()
    N, H, W, Kc, Cc = 2, 14, 14, 256, 128
    if Cc % tile[1]:
        pytest.skip("tile wider than C")
    torch.manual_seed(6)
    g = torch.randn(N, H, W, Kc, device=dev).bfloat16()
    y = torch.randn_like(g)
    coeff = torch.randn(3 * Kc, device=dev) * 0.5
    wt = (torch.randn(Cc, Kc, device=dev) / math.sqrt(Kc)).bfloat16()
    ybn = torch.randn(N, H, W, Cc, device=dev).bfloat16()
    mean, inv = torch.randn(Cc, device=dev) * 0.1, torch.rand(Cc, device=dev) + 0.5
    sc, sh = torch.rand(Cc, device=dev) + 0.5, torch.randn(Cc, device=dev) * 0.1
    add = torch.randn_like(ybn)
    mbits = k.pack_mask_bits(torch.randn_like(ybn))

    def run(dma):
        s1 = k.new_stats(Cc, dev)
        dx = torch.empty(N, H, W, Cc, device=dev, dtype=torch.bfloat16)
        dy_out = torch.full_like(g, float("nan"))
        kw = dict(bwd_y=y, bwd_coeff=coeff, dy_out=dy_out, tile=(*tile, dma))
        if variant == "epi2":
            kw["epilogue"] = k.BNBwdEpilogue(k.MASK_Y, ybn, mean, inv, s1, scale=sc, shift=sh)
        elif variant == "epi1_acc":
            kw.update(epilogue=k.BNBwdEpilogue(k.MASK_OUT, ybn, mean, inv, s1, mbits=mbits), addsrc=add)
        k.conv_dgrad(g, wt, dx, R=1, S=1, stride=1, pad=0, **kw)
        return dx, s1, dy_out

    _same(run(0), run(1), (tile, variant))
