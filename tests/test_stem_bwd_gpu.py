"""Fused stem backward (csrc/stem_bwd.hip) == max-pool backward + BN-backward apply + stem weight
gradient, against a plain PyTorch fp32 reference and against the unfused kernels."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

dev = "cuda"


def K():
    from dbx_distributed_pytorch_examples_amd.ops import kernels
    return kernels


def relerr(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _setup(N, HI, seed=0):
    """A real stem forward (conv 7x7/2 -> y0, BN scale/shift, 3x3/2 max-pool with argmax) so the
    argmax bytes are consistent with y0, plus a random pooled gradient and BN-backward coefficients."""
    k = K()
    torch.manual_seed(seed)
    x4 = torch.zeros(N, HI, HI, 4, device=dev, dtype=torch.bfloat16)
    x4[..., :3] = torch.randn(N, HI, HI, 3, device=dev).bfloat16()
    w = torch.zeros(64, 8, 8, 4, device=dev)
    w[:, :7, :7, :3] = torch.randn(64, 7, 7, 3, device=dev) * 0.1
    w16 = w.view(64, 256).bfloat16()
    H = (HI + 6 - 7) // 2 + 1
    y0 = torch.empty(N, H, H, 64, device=dev, dtype=torch.bfloat16)
    k.conv_stem_fwd(x4, w16, y0, R=7, S=7, stride=2, pad=3)
    sc, sh = torch.rand(64, device=dev) + 0.5, torch.randn(64, device=dev) * 0.2
    P = (H + 2 - 3) // 2 + 1
    p0 = torch.empty(N, P, P, 64, device=dev, dtype=torch.bfloat16)
    arg = torch.empty(N, P, P, 64, device=dev, dtype=torch.uint8)
    k.maxpool_fwd(y0, p0, arg, K=3, stride=2, pad=1, scale=sc, shift=sh, relu=True)
    dp = torch.randn(N, P, P, 64, device=dev).bfloat16()
    coeff = torch.randn(3 * 64, device=dev) * 0.3
    return x4, y0, sc, sh, dp, arg, coeff


def _fused(x4, y0, sc, sh, dp, arg, coeff):
    k = K()
    dw = torch.full((64, 256), float("nan"), device=dev)
    ws = torch.empty(600 * 64 * 256, device=dev)
    k.stem_bwd_fused(dp, arg, y0, sc, sh, coeff, x4, dw, ws)
    torch.cuda.synchronize()
    return dw


@pytest.mark.parametrize("N,HI", [(2, 32), (4, 224), (16, 224)])
def test_stem_bwd_fused_matches_unfused(N, HI):
    k = K()
    x4, y0, sc, sh, dp, arg, coeff = _setup(N, HI)
    dw = _fused(x4, y0, sc, sh, dp, arg, coeff)
    dy = torch.empty_like(y0)
    k.pool_bn_bwd_apply(dp, arg, y0, sc, sh, coeff, dy, K=3, stride=2, pad=1)
    dw_u = torch.empty(64, 256, device=dev)
    ws = torch.empty(600 * 64 * 256, device=dev)
    k.conv_wgrad(dy, x4, dw_u, ws, R=7, S=7, stride=2, pad=3, stem=True)
    torch.cuda.synchronize()
    assert torch.isfinite(dw).all()
    assert relerr(dw, dw_u) < 1e-3
    # padded taps (s = 7, channel 3) carry no gradient
    assert dw.view(64, 8, 8, 4)[:, :, 7].abs().max().item() == 0.0
    assert dw.view(64, 8, 8, 4)[..., 3].abs().max().item() == 0.0


def test_stem_bwd_fused_matches_fp32_reference():
    x4, y0, sc, sh, dp, arg, coeff = _setup(2, 64, seed=3)
    dw = _fused(x4, y0, sc, sh, dp, arg, coeff)
    # fp32 reference: max-pool backward through autograd on the BN+ReLU output (rounded to bf16 as the
    # forward kernel pools it), the ReLU mask, the BN-backward apply, the 7x7/2 stem weight gradient
    t = y0.float() * sc + sh
    act = torch.relu(t).bfloat16().float().permute(0, 3, 1, 2).requires_grad_(True)
    F.max_pool2d(act, 3, 2, 1).backward(dp.float().permute(0, 3, 1, 2))
    g = act.grad.permute(0, 2, 3, 1) * (t > 0)
    k1, k2, k3 = coeff.view(3, 64)
    dy = (k1 * g + k2 * y0.float() + k3).bfloat16().float().permute(0, 3, 1, 2)
    wref = torch.nn.grad.conv2d_weight(x4.float().permute(0, 3, 1, 2)[:, :3], (64, 3, 7, 7), dy, stride=2, padding=3)
    got = dw.view(64, 8, 8, 4)[:, :7, :7, :3].permute(0, 3, 1, 2)
    assert relerr(got, wref) < 2e-2


def test_stem_bwd_fused_deterministic():
    args = _setup(8, 224, seed=5)
    assert torch.equal(_fused(*args), _fused(*args))


def test_native_step_stem_fused_vs_unfused(monkeypatch, engine):
    """One eager ResNet-50 step at 224: fused stem backward (opt-in, fuse_stem_bwd=1) ==
    pool_bn_bwd_apply + stem wgrad."""
    from dbx_distributed_pytorch_examples_amd.engine.native_trainer import NativeTrainer, OptimConfig
    from dbx_distributed_pytorch_examples_amd.models import resnet50

    torch.manual_seed(5)
    img = torch.randint(0, 256, (2, 224, 224, 3), dtype=torch.uint8, device=dev)
    lab = torch.randint(0, 1000, (2,), device=dev)
    grads = []
    for flag in ("1", "0"):
        engine(fuse_stem_bwd=flag)
        torch.manual_seed(0)
        tr = NativeTrainer(resnet50(num_classes=1000), 2, (224, 224), torch.device(dev), optim=OptimConfig(lr=0.0),
                           use_graphs=False)
        tr.step(img, lab)
        torch.cuda.synchronize()
        grads.append(tr.prog.grad.clone())
    st = tr.prog.stem
    a, b = grads[0][st.off:st.off + st.numel], grads[1][st.off:st.off + st.numel]
    assert relerr(a, b) < 1e-3
    assert relerr(grads[0], grads[1]) < 1e-2


@pytest.mark.parametrize("N,HI", [(2, 32), (8, 224)])
def test_stem_wgrad_tile_matches_generic(N, HI):
    """The 64 x 256-tile stem weight gradient (stem_bwd.hip, plain mode; conv_wgrad's default for the
    64-channel stem) == the generic wgrad kernel's STEM mode (tile=(64, 128))."""
    k = K()
    torch.manual_seed(2)
    x4 = torch.zeros(N, HI, HI, 4, device=dev, dtype=torch.bfloat16)
    x4[..., :3] = torch.randn(N, HI, HI, 3, device=dev).bfloat16()
    H = (HI + 6 - 7) // 2 + 1
    dy = torch.randn(N, H, H, 64, device=dev).bfloat16()
    ws = torch.empty(600 * 64 * 256, device=dev)
    a, b = torch.empty(64, 256, device=dev), torch.empty(64, 256, device=dev)
    k.conv_wgrad(dy, x4, a, ws, R=7, S=7, stride=2, pad=3, stem=True)
    k.conv_wgrad(dy, x4, b, ws, R=7, S=7, stride=2, pad=3, stem=True, tile=(64, 128))
    torch.cuda.synchronize()
    assert relerr(a, b) < 1e-4
    assert a.view(64, 8, 8, 4)[:, :, 7].abs().max().item() == 0.0
