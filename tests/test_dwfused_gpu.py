"""Fused bottleneck-conv3 backward (csrc/conv_dwfused.hip) against a plain PyTorch fp32 reference
of the same math, against the unfused kernel schedule, and inside the native ResNet-50 step."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

dev = "cuda"


def K():
    from dbx_distributed_pytorch_examples_amd.ops import kernels
    return kernels


def relerr(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _inputs(N, H, W, seed=7, Cc=64, Kc=256):
    torch.manual_seed(seed)
    g = torch.randn(N, H, W, Kc, device=dev).bfloat16()
    y3 = torch.randn(N, H, W, Kc, device=dev).bfloat16()
    coeff = torch.randn(3 * Kc, device=dev) * 0.5
    wt = (torch.randn(Cc, Kc, device=dev) / math.sqrt(Kc)).bfloat16()
    y2 = torch.randn(N, H, W, Cc, device=dev).bfloat16()
    sc, sh = torch.rand(Cc, device=dev) + 0.5, torch.randn(Cc, device=dev) * 0.3
    mean, inv = torch.randn(Cc, device=dev) * 0.1, torch.rand(Cc, device=dev) + 0.5
    return g, y3, coeff, wt, y2, sc, sh, mean, inv


def _run_fused(g, y3, coeff, wt, y2, sc, sh, mean, inv, cus=0):
    k = K()
    N, H, W, Kc = g.shape
    Cc = y2.shape[-1]
    da = torch.full((N, H, W, Cc), float("nan"), device=dev, dtype=torch.bfloat16)
    dw = torch.full((Kc, Cc), float("nan"), device=dev)
    st = k.new_stats(Cc, dev)
    ws = torch.empty((1024 + 64) * Kc * Cc, device=dev)
    k.conv_dwfused(g, y3, coeff, wt, y2, sc, sh, mean, inv, st, da, dw, ws, cus=cus)
    torch.cuda.synchronize()
    return da, dw, st.view(-1, 2, Cc).sum(0)


@pytest.mark.parametrize("nhw,ck", [((2, 16, 16), (64, 256)), ((4, 56, 56), (64, 256)), ((48, 56, 56), (64, 256)),
                                    ((1, 8, 8), (128, 512)), ((4, 28, 28), (128, 512)), ((24, 28, 28), (128, 512)),
                                    ((64, 28, 28), (128, 512))])
def test_dwfused_matches_fp32_reference(nhw, ck):
    """56x56-stage variant (128-pixel tiles): 4 / 98 / 1176 tiles; 28x28-stage variant (64-pixel
    tiles, one workgroup per CU): 1 / 49 / 294 / 784 tiles (grid below / above the resident capacity)."""
    N, H, W = nhw
    g, y3, coeff, wt, y2, sc, sh, mean, inv = _inputs(N, H, W, Cc=ck[0], Kc=ck[1])
    da, dw, st = _run_fused(g, y3, coeff, wt, y2, sc, sh, mean, inv)
    Kc, Cc = g.shape[-1], y2.shape[-1]
    k1, k2, k3 = coeff.view(3, Kc)
    dy = (g.float() * k1 + y3.float() * k2 + k3).bfloat16().float().reshape(-1, Kc)
    t = (y2.float() * sc + sh).reshape(-1, Cc)
    a2 = torch.relu(t).bfloat16().float()
    raw = (dy @ wt.float().t()).bfloat16().float()
    da_ref = (raw * (t > 0)).bfloat16().float()
    dw_ref = dy.t() @ a2
    s_ref = da_ref.sum(0)
    q_ref = (da_ref * ((y2.float().reshape(-1, Cc) - mean) * inv)).sum(0)
    assert torch.isfinite(da.float()).all() and torch.isfinite(dw).all()
    assert relerr(da.reshape(-1, Cc), da_ref) < 1e-2
    assert relerr(dw, dw_ref) < 5e-3
    M = N * H * W
    assert ((st[0].float() - s_ref).abs() / (s_ref.abs() + 0.01 * M)).max().item() < 2e-2
    assert ((st[1].float() - q_ref).abs() / (q_ref.abs() + 0.01 * M)).max().item() < 2e-2


@pytest.mark.parametrize("nhw,ck", [((8, 56, 56), (64, 256)), ((16, 28, 28), (128, 512))])
def test_dwfused_matches_unfused_kernels(nhw, ck):
    """== BN-backward apply folded into the MASK_Y dgrad (stores dy3 and a2) + the weight gradient."""
    k = K()
    Cc, Kc = ck
    g, y3, coeff, wt, y2, sc, sh, mean, inv = _inputs(*nhw, seed=11, Cc=Cc, Kc=Kc)
    da, dw, st = _run_fused(g, y3, coeff, wt, y2, sc, sh, mean, inv)
    st_u = k.new_stats(Cc, dev)
    da_u = torch.empty_like(da)
    dy3 = torch.empty_like(g)
    act = torch.empty_like(y2)
    e = k.BNBwdEpilogue(k.MASK_Y, y2, mean, inv, st_u, scale=sc, shift=sh, act_out=act)
    k.conv_dgrad(g, wt, da_u, R=1, S=1, stride=1, pad=0, epilogue=e, bwd_y=y3, bwd_coeff=coeff, dy_out=dy3)
    dw_u = torch.empty(Kc, Cc, device=dev)
    ws = torch.empty(64 * Kc * Cc * 4, device=dev)
    k.conv_wgrad(dy3, act, dw_u, ws, R=1, S=1, stride=1, pad=0)
    torch.cuda.synchronize()
    assert relerr(da, da_u) < 2e-3
    assert relerr(dw, dw_u) < 1e-3
    b = st_u.view(-1, 2, Cc).sum(0)
    assert ((st - b).abs() / (b.abs() + 1.0)).max().item() < 1e-2


@pytest.mark.parametrize("nhw,ck", [((16, 56, 56), (64, 256)), ((16, 28, 28), (128, 512))])
def test_dwfused_deterministic(nhw, ck):
    """Fixed tile -> workgroup assignment, fixed-order slab reduction, fp64 moment atomics."""
    args = _inputs(*nhw, seed=3, Cc=ck[0], Kc=ck[1])
    a = _run_fused(*args)
    b = _run_fused(*args)
    for x, y in zip(a, b):
        assert torch.equal(x, y)


@pytest.mark.parametrize("nhw,ck", [((16, 56, 56), (64, 256)), ((16, 28, 28), (128, 512))])
def test_dwfused_cu_span(nhw, ck):
    """``cus`` (the persistent grid spans only 128 CUs): the same data gradient bit for bit (it does not
    depend on the tile -> workgroup assignment), the weight gradient summed over fewer slabs."""
    args = _inputs(*nhw, seed=5, Cc=ck[0], Kc=ck[1])
    da, dw, st = _run_fused(*args)
    da2, dw2, st2 = _run_fused(*args, cus=128)
    assert torch.equal(da, da2)
    assert relerr(dw2, dw) < 1e-5
    assert ((st2 - st).abs() / (st.abs() + 1.0)).max().item() < 1e-6


def test_native_step_fused_vs_unfused(monkeypatch, engine):
    """One eager ResNet-50 step at 224 (stage-1 / stage-2 conv3s take the fused kernel) == the unfused
    schedule."""
    from dbx_distributed_pytorch_examples_amd.engine.native_trainer import NativeTrainer, OptimConfig
    from dbx_distributed_pytorch_examples_amd.models import resnet50

    torch.manual_seed(5)
    img = torch.randint(0, 256, (2, 224, 224, 3), dtype=torch.uint8, device=dev)
    lab = torch.randint(0, 1000, (2,), device=dev)
    grads = []
    engine(fuse_dw_min_tiles="0")  # batch 2: fuse regardless of tiles per workgroup
    for flag in ("1", "0"):
        engine(fuse_dw=flag)
        torch.manual_seed(0)
        tr = NativeTrainer(resnet50(num_classes=1000), 2, (224, 224), torch.device(dev), optim=OptimConfig(lr=0.0),
                           use_graphs=False)
        assert (tr.prog.ws_dw is not None) == (flag == "1")
        tr.step(img, lab)
        torch.cuda.synchronize()
        grads.append(tr.prog.grad.clone())
    assert relerr(grads[0], grads[1]) < 2e-2
    # the fused conv3 weight gradients themselves
    tr_names = [n for n, _, _ in tr.prog.param_ranges]
    for name, off, n in tr.prog.param_ranges:
        if name.startswith(("layer1.", "layer2.")) and name.endswith("conv3.weight"):
            assert relerr(grads[0][off:off + n], grads[1][off:off + n]) < 2e-2, name
    assert any(n.startswith("layer1.") for n in tr_names)
