"""Weights-stationary 3x3 patch kernel (csrc/conv_patch3.hip) vs the implicit-GEMM path.

Same tap order, same MFMA operand roles and fp32 accumulation order as the implicit GEMM, so the
conv outputs (and the MASK_Y epilogue's masked gradient / BN-output write-back) must be
bit-identical; the BN statistics are sums of different per-tile fp32 partials (448-row tiles
instead of 128) and are compared with a tolerance. The implicit GEMM itself is checked against
fp32 PyTorch in test_kernels_gpu.py.
"""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
dev = "cuda"


def K():
    from dbx_distributed_pytorch_examples_amd.ops import kernels
    return kernels


@pytest.fixture(autouse=True)
def _no_splitk(engine):
    """These compare kernels bit for bit against the four-wave implicit-GEMM launch, which splits the K
    loop of few-tile launches (splitk_wgs; its own tests: test_splitk_gpu.py): compare unsplit launches."""
    engine(splitk_wgs=0)


def _close_stats(a, b, count):
    a, b = a.view(-1, 2, 64).sum(0), b.view(-1, 2, 64).sum(0)
    return ((a - b).abs() / (b.abs() + count * 1e-3)).max().item()


@pytest.mark.parametrize("N,H", [(2, 56), (3, 16), (1, 8)])
@pytest.mark.parametrize("prologue", [True, False])
def test_patch3_fwd_matches_igemm(N, H, prologue):
    k = K()
    torch.manual_seed(7)
    W, C = 56, 64
    assert k.patch3_supported(C, C, 3, 3, 1, 1, H, W)
    x = torch.randn(N, H, W, C, device=dev).bfloat16()
    w = (torch.randn(C, 9 * C, device=dev) / math.sqrt(9 * C)).bfloat16()
    sc = sh = None
    if prologue:
        sc, sh = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1
    outs = []
    for tile in ((128, 64), "patch_r", "patch_s"):
        y = torch.full((N, H, W, C), float("nan"), device=dev, dtype=torch.bfloat16)
        st = k.new_stats(C, dev)
        k.conv_fwd(x, w, y, R=3, S=3, stride=1, pad=1, stats=st, in_scale=sc, in_shift=sh, tile=tile)
        outs.append((y, st))
    torch.cuda.synchronize()
    for o in outs[1:]:
        assert torch.equal(outs[0][0], o[0])
        assert _close_stats(o[1], outs[0][1], N * H * W) < 1e-5


@pytest.mark.parametrize("N,H", [(2, 56), (3, 16)])
@pytest.mark.parametrize("epi", [None, "mask_y"])
def test_patch3_dgrad_matches_igemm(N, H, epi):
    k = K()
    torch.manual_seed(8)
    W, C = 56, 64
    w = (torch.randn(C, 3, 3, C, device=dev) / math.sqrt(9 * C)).bfloat16()
    wt = w.permute(3, 1, 2, 0).contiguous().view(C, -1)
    dy = torch.randn(N, H, W, C, device=dev).bfloat16()
    ybn = torch.randn(N, H, W, C, device=dev).bfloat16()
    sc, sh = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1
    mean, inv = torch.randn(C, device=dev) * 0.1, torch.rand(C, device=dev) + 0.5
    outs = []
    for tile in ((256, 64), "patch_r", "patch_s"):
        dx = torch.full((N, H, W, C), float("nan"), device=dev, dtype=torch.bfloat16)
        st = k.new_stats(C, dev)
        act = torch.full_like(dx, float("nan"))
        e = None
        if epi:
            e = k.BNBwdEpilogue(k.MASK_Y, ybn, mean, inv, st, scale=sc, shift=sh, act_out=act)
        k.conv_dgrad(dy, wt, dx, R=3, S=3, stride=1, pad=1, epilogue=e, tile=tile)
        outs.append((dx, st, act))
    torch.cuda.synchronize()
    for o in outs[1:]:
        assert torch.equal(outs[0][0], o[0])
        if epi:
            assert torch.equal(outs[0][2], o[2])
            assert _close_stats(o[1], outs[0][1], N * H * W) < 1e-5


def test_patch3_default_routing_and_fallbacks():
    """Eligible convs take the patch kernel by default; an addend / stride / other width falls back."""
    k = K()
    assert not k.patch3_supported(64, 64, 3, 3, 2, 1, 56, 56)
    assert not k.patch3_supported(128, 128, 3, 3, 1, 1, 28, 28)
    assert not k.patch3_supported(64, 64, 3, 3, 1, 1, 12, 56)
    torch.manual_seed(9)
    x = torch.randn(1, 8, 56, 64, device=dev).bfloat16()
    w = (torch.randn(64, 9 * 64, device=dev) / 24).bfloat16()
    y1, y2 = torch.empty_like(x), torch.empty_like(x)
    k.conv_fwd(x, w, y1, R=3, S=3, stride=1, pad=1)
    k.conv_fwd(x, w, y2, R=3, S=3, stride=1, pad=1, tile="patch")
    assert torch.equal(y1, y2)
    with pytest.raises(ValueError):
        k.conv_fwd(torch.randn(1, 8, 28, 64, device=dev).bfloat16(), w, torch.empty(1, 8, 28, 64, device=dev).bfloat16(),
                   R=3, S=3, stride=1, pad=1, tile="patch")


@pytest.mark.parametrize("N,H", [(2, 224), (1, 96)])
def test_stem_patch_vs_fp32(N, H):
    """Stem patch kernel (7x7/2 on the NHWC4 image, width 224) vs fp32 torch, and vs the implicit
    GEMM stem (same products, different order inside a K step: close, not bit-exact)."""
    k = K()
    W = 224
    torch.manual_seed(10)
    img = torch.randn(N, H, W, 3, device=dev)
    x4 = torch.zeros(N, H, W, 4, device=dev)
    x4[..., :3] = img
    x4 = x4.bfloat16()
    w = torch.randn(64, 7, 7, 3, device=dev) * 0.05
    ws_ = torch.zeros(64, 8, 8, 4, device=dev)
    ws_[:, :7, :7, :3] = w
    w16s = ws_.bfloat16().view(64, 256)
    OH, OW = k.conv_out_hw(H, W, 7, 7, 2, 3)
    assert k.stem_patch_supported(H, W, 64, 7, 7, 2, 3)
    outs = []
    for patch in (True, False):
        out = torch.full((N, OH, OW, 64), float("nan"), device=dev, dtype=torch.bfloat16)
        st = k.new_stats(64, dev)
        k.conv_stem_fwd(x4, w16s, out, stats=st, patch=patch)
        outs.append((out, st))
    torch.cuda.synchronize()
    ref = F.conv2d(x4[..., :3].float().permute(0, 3, 1, 2), ws_.bfloat16().float()[:, :7, :7, :3].permute(0, 3, 1, 2),
                   stride=2, padding=3).permute(0, 2, 3, 1)
    out, st = outs[0]
    assert not torch.isnan(out.float()).any()
    assert ((out.float() - ref).norm() / ref.norm()).item() < 1e-2
    assert (out.float() - outs[1][0].float()).abs().max().item() <= 0.02 * ref.abs().max().item()
    s = st.view(-1, 2, 64).sum(0)
    o = out.float().view(-1, 64)
    assert ((s[0] - o.sum(0)).abs() / (o.abs().sum(0) + 1)).max().item() < 1e-3
    assert ((s[1] - (o * o).sum(0)).abs() / ((o * o).sum(0) + 1)).max().item() < 1e-3


@pytest.mark.parametrize("N,H", [(2, 56), (3, 16), (1, 8)])
def test_wgrad_patch3_vs_fp32(N, H):
    """3x3 patch weight gradient (per-workgroup fp32 slabs + ordered reduction) vs fp32 torch and
    vs the implicit-GEMM wgrad; also the accumulate / scale arguments."""
    k = K()
    torch.manual_seed(11)
    W, C = 56, 64
    x = torch.randn(N, H, W, C, device=dev).bfloat16()
    dy = torch.randn(N, H, W, C, device=dev).bfloat16()
    ws = torch.empty(400 * C * 9 * C, device=dev)
    ref = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), (C, C, 3, 3), dy.float().permute(0, 3, 1, 2),
                                      stride=1, padding=1).permute(0, 2, 3, 1).reshape(C, -1)
    dw_p = torch.full((C, 9 * C), float("nan"), device=dev)
    k.conv_wgrad(dy, x, dw_p, ws, R=3, S=3, stride=1, pad=1, tile="patch")
    dw_i = torch.empty_like(dw_p)
    k.conv_wgrad(dy, x, dw_i, ws, R=3, S=3, stride=1, pad=1, tile=(64, 64))
    torch.cuda.synchronize()
    assert ((dw_p - ref).norm() / ref.norm()).item() < 1e-4
    assert ((dw_p - dw_i).norm() / ref.norm()).item() < 1e-4
    base = torch.randn_like(dw_p)
    dw2 = base.clone()
    k.conv_wgrad(dy, x, dw2, ws, R=3, S=3, stride=1, pad=1, tile="patch", scale=0.5, accumulate=True)
    assert ((dw2 - (base + 0.5 * ref)).norm() / ref.norm()).item() < 1e-4
    # deterministic: a second run is bit-identical
    dw3 = torch.empty_like(dw_p)
    k.conv_wgrad(dy, x, dw3, ws, R=3, S=3, stride=1, pad=1, tile="patch")
    assert torch.equal(dw3, dw_p)
