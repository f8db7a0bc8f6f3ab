"""N-sweep 1x1 convs (csrc/conv_sweep.hip, tile code dma 8). The BN-prologue forward: against the fp32 PyTorch
reference of relu(x*scale + shift) conv 1x1, and bit-identical (outputs and BN statistics) to the
128 x 256 implicit-GEMM tile it replaces -- same MFMA order, same per-tile statistics partials --
including rows past M, the in-launch BN finalize and graph replays."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

dev = "cuda"


def K():
    from dbx_distributed_pytorch_examples_amd.ops import kernels
    return kernels


def relerr(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def _run(k, x, w, sc, sh, tile, stats=True, fin=None):
    N, H, W, IC = x.shape
    OC = w.shape[0]
    out = torch.empty(N, H, W, OC, device=dev, dtype=torch.bfloat16)
    st = k.new_stats(OC, dev) if stats else None
    k.conv_fwd(x, w, out, R=1, S=1, stride=1, pad=0, stats=st, in_scale=sc, in_shift=sh, relu_in=True,
               tile=tile, fin=fin)
    return out, st


# N, H, IC, OC: ResNet-50 conv3 expansions at small batch (rows past M in the last 128-row block for
# the odd sizes), every K block count of the kernel (64..256 channels)
CASES = [(6, 14, 256, 1024), (5, 28, 128, 512), (3, 28, 64, 256 * 3), (7, 14, 192, 512), (2, 7, 256, 1024)]


@pytest.mark.parametrize("case", CASES)
def test_sweep_matches_igemm_and_reference(case):
    k = K()
    N, H, IC, OC = case
    torch.manual_seed(0)
    x = torch.randn(N, H, H, IC, device=dev).bfloat16()
    w = (torch.randn(OC, IC, device=dev) / math.sqrt(IC)).bfloat16()
    sc = torch.rand(IC, device=dev) + 0.5
    sh = torch.randn(IC, device=dev) * 0.1
    xe = torch.relu(x.float() * sc + sh).bfloat16().float()
    ref = (xe.view(-1, IC) @ w.float().t()).view(N, H, H, OC)
    o0, s0 = _run(k, x, w, sc, sh, (128, 256, 1))
    o1, s1 = _run(k, x, w, sc, sh, (128, 256, 8))
    torch.cuda.synchronize()
    assert relerr(o1, ref) < 1e-2
    assert torch.equal(o1, o0)
    assert torch.equal(s1, s0)
    ob = o1.float().view(-1, OC)
    tot = s1.view(-1, 2, OC).sum(0)
    assert torch.allclose(tot[0], ob.sum(0).double(), rtol=1e-4, atol=1e-2)
    assert torch.allclose(tot[1], (ob * ob).sum(0).double(), rtol=1e-4, atol=1e-2)
    o2, _ = _run(k, x, w, sc, sh, (128, 256, 8), stats=False)
    assert torch.equal(o2, o0)


def test_sweep_selected_for_headline_shapes(engine):
    """The engine picks the sweep kernel for the b1024 conv3 expansions at 28 / 14 and not for the
    one-sub-tile, tail-prologue or few-block launches."""
    k = K()
    engine(sweep_fwd=True)
    cus = k.num_cus()
    assert k.sweep_fwd_ok(1024 * 14 * 14, 256, 1024, 1, 1, 1, 0, True, True, True)
    assert k.sweep_fwd_ok(1024 * 28 * 28, 128, 512, 1, 1, 1, 0, True, True, True)
    assert k.sweep_fwd_ok(1024 * 56 * 56, 64, 256, 1, 1, 1, 0, True, True, True)         # one sub-tile
    assert not k.sweep_fwd_ok(1024 * 56 * 56, 64, 64, 1, 1, 1, 0, True, True, True)      # OC < 256
    assert not k.sweep_fwd_ok(1024 * 7 * 7, 512, 2048, 1, 1, 1, 0, True, True, True)     # K > 256
    assert not k.sweep_fwd_ok(1024 * 14 * 14, 256, 1024, 1, 1, 1, 0, True, False, True)  # tail prologue
    assert not k.sweep_fwd_ok(512 * 4 * 4, 256, 1024, 1, 1, 1, 0, True, True, True)      # few blocks
    assert not k.sweep_fwd_ok(128 * 4 * cus, 256, 1024, 3, 3, 1, 1, True, True, True)    # 3x3
    engine(sweep_fwd=False)
    assert not k.sweep_fwd_ok(1024 * 14 * 14, 256, 1024, 1, 1, 1, 0, True, True, True)


def test_sweep_in_launch_finalize_and_graph_replay():
    """The in-launch BN finalize (bn_fin_tail over the sub-tiles' arrivals) gives the standalone
    finalize's scale / shift; a captured sweep launch replays to the same bits."""
    k = K()
    N, H, IC, OC = 9, 14, 256, 1024
    torch.manual_seed(1)
    x = torch.randn(N, H, H, IC, device=dev).bfloat16()
    w = (torch.randn(OC, IC, device=dev) / math.sqrt(IC)).bfloat16()
    sc = torch.rand(IC, device=dev) + 0.5
    sh = torch.randn(IC, device=dev) * 0.1
    gamma, beta = torch.rand(OC, device=dev) + 0.5, torch.randn(OC, device=dev)
    res = []
    for tile in ((128, 256, 1), (128, 256, 8)):
        st = k.new_stats(OC, dev)
        bufs = [torch.zeros(OC, device=dev) for _ in range(6)]
        fin = k.BnFin(k.BnFin.FWD, st, N * H * H, gamma=gamma, beta=beta, eps=1e-5, momentum=0.1,
                      running_mean=bufs[0], running_var=bufs[1], scale=bufs[2], shift=bufs[3], mean=bufs[4],
                      invstd=bufs[5])
        out = torch.empty(N, H, H, OC, device=dev, dtype=torch.bfloat16)
        k.conv_fwd(x, w, out, R=1, S=1, stride=1, pad=0, stats=st, in_scale=sc, in_shift=sh, tile=tile, fin=fin)
        torch.cuda.synchronize()
        res.append((out, st, bufs))
    (o0, s0, b0), (o1, s1, b1) = res
    assert torch.equal(o0, o1) and torch.equal(s0, s1)
    for u, v in zip(b0, b1):  # the in-launch finalize: same scale / shift / moments / running stats
        assert torch.equal(u, v)
    assert b1[2].abs().sum() > 0
    # graph replay of the sweep launch
    out = torch.empty_like(o1)
    stg = k.new_stats(OC, dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            k.conv_fwd(x, w, out, R=1, S=1, stride=1, pad=0, stats=stg, in_scale=sc, in_shift=sh, tile=(128, 256, 8))
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(3):
        out.zero_()
        stg.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, o1) and torch.equal(stg, s1)


# N, H, K (conv1 output channels = the dgrad's staged channels), Cc (its input channels): the
# bottleneck conv1 data gradients (rows past M in the last block for the odd sizes)
DCASES = [(6, 14, 256, 1024), (5, 28, 128, 512), (3, 56, 64, 256), (7, 14, 192, 512)]


@pytest.mark.parametrize("case", DCASES)
@pytest.mark.parametrize("variant", ["epi1", "epi1_ds", "accum_only"])
def test_sweep_dgrad_matches_igemm(case, variant):
    """Folded BN1-backward dgrad + block-input addend + the previous block's MASK_OUT epilogue (and its
    downsample BN's second statistic): dx, the stored dy and both statistics bit-identical to the
    128 x 256 implicit-GEMM tile; dx against the fp32 reference."""
    k = K()
    N, H, Kc, Cc = case
    torch.manual_seed(2)
    g = torch.randn(N, H, H, Kc, device=dev).bfloat16()
    yb = torch.randn(N, H, H, Kc, device=dev).bfloat16()
    coeff = torch.randn(3, Kc, device=dev) * 0.5
    wt = (torch.randn(Cc, Kc, device=dev) / math.sqrt(Kc)).bfloat16()
    add = torch.randn(N, H, H, Cc, device=dev).bfloat16()
    ybn = torch.randn(N, H, H, Cc, device=dev).bfloat16()
    ybn2 = torch.randn(N, H, H, Cc, device=dev).bfloat16()
    mask = torch.randn(N, H, H, Cc, device=dev) > 0
    mb = k.pack_mask_bits(mask)
    m1, i1 = torch.randn(Cc, device=dev) * 0.1, torch.rand(Cc, device=dev) + 0.5
    m2, i2 = torch.randn(Cc, device=dev) * 0.1, torch.rand(Cc, device=dev) + 0.5
    outs = []
    for tile in ((128, 256, 1), (128, 256, 8)):
        dx = torch.empty(N, H, H, Cc, device=dev, dtype=torch.bfloat16)
        dyo = torch.empty_like(g)
        s1, s2 = k.new_stats(Cc, dev), k.new_stats(Cc, dev)
        epi = None
        if variant != "accum_only":
            epi = k.BNBwdEpilogue(k.MASK_OUT, ybn, m1, i1, s1, mbits=mb,
                                  **(dict(ybn2=ybn2, mean2=m2, inv2=i2, stats2=s2) if variant == "epi1_ds" else {}))
        k.conv_dgrad(g, wt, dx, R=1, S=1, stride=1, pad=0, tile=tile, addsrc=add, epilogue=epi, bwd_y=yb,
                     bwd_coeff=coeff, dy_out=dyo)
        torch.cuda.synchronize()
        outs.append((dx, dyo, s1, s2))
    (a0, b0, c0, d0), (a1, b1, c1, d1) = outs
    assert torch.equal(b1, b0), "stored BN-backward operand"
    assert torch.equal(a1, a0), "data gradient"
    assert torch.equal(c1, c0) and torch.equal(d1, d0), "statistics"
    # fp32 reference of the data gradient
    dyr = (g.float() * coeff[0] + yb.float() * coeff[1] + coeff[2]).bfloat16().float()
    assert relerr(b1, dyr) < 1e-2
    ref = (dyr.view(-1, Kc) @ wt.float().t()).view(N, H, H, Cc) + add.float()
    if variant != "accum_only":
        ref = ref * mask
    assert relerr(a1, ref) < 1e-2


def test_sweep_dgrad_selected(engine):
    k = K()
    engine(sweep_dgrad=True)
    assert k.sweep_dgrad_ok(1024 * 14 * 14, 256, 1024, 1, 1, 1, 0, True, 1, k.MASK_OUT)
    assert k.sweep_dgrad_ok(1024 * 56 * 56, 64, 256, 1, 1, 1, 0, True, 1, 0)
    assert not k.sweep_dgrad_ok(1024 * 14 * 14, 1024, 256, 1, 1, 1, 0, True, 1, k.MASK_Y)  # K > 256, MASK_Y
    assert not k.sweep_dgrad_ok(1024 * 28 * 28, 256, 512, 1, 1, 1, 0, True, 2, k.MASK_OUT)  # subsampled addend
    assert not k.sweep_dgrad_ok(1024 * 14 * 14, 256, 1024, 1, 1, 1, 0, False, 1, k.MASK_OUT)  # not folded
    engine(sweep_dgrad=False)
    assert not k.sweep_dgrad_ok(1024 * 14 * 14, 256, 1024, 1, 1, 1, 0, True, 1, k.MASK_OUT)
