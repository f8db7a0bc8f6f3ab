"""Numerics of every HIP kernel against a plain PyTorch fp32 reference of the same op.

Shapes come from the ResNet conv tables in SURVEY.md §2.4 / Appendix A at small batch.
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


def relerr(a, b):
    a = a.float()
    b = b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


def nchw(x):
    return x.permute(0, 3, 1, 2).contiguous()


CONV_CASES = [
    # N, H, W, IC, OC, R, stride, pad
    (2, 14, 14, 64, 64, 3, 1, 1),
    (2, 14, 14, 64, 256, 1, 1, 0),
    (2, 14, 14, 256, 64, 1, 1, 0),
    (2, 14, 14, 128, 128, 3, 2, 1),
    (2, 14, 14, 256, 512, 1, 2, 0),
    (3, 7, 7, 512, 512, 3, 1, 1),
    (4, 9, 9, 64, 128, 3, 2, 1),
    (1, 5, 5, 128, 64, 3, 1, 1),
    # small maps: the launches visit only the taps that touch data (fwd_taps / dgrad_phases)
    (8, 1, 1, 512, 512, 3, 1, 1),
    (8, 2, 2, 256, 512, 3, 2, 1),
    (8, 2, 2, 256, 256, 3, 1, 1),
    (4, 1, 2, 128, 64, 3, 1, 1),
]


@pytest.mark.parametrize("case", CONV_CASES)
@pytest.mark.parametrize("prologue", [False, True])
def test_conv_fwd(case, prologue):
    k = K()
    N, H, W, IC, OC, R, st, pad = case
    torch.manual_seed(0)
    x = torch.randn(N, H, W, IC, device=dev).bfloat16()
    w = (torch.randn(OC, R, R, IC, device=dev) / math.sqrt(IC * R * R)).bfloat16()
    OH, OW = k.conv_out_hw(H, W, R, R, st, pad)
    out = torch.empty(N, OH, OW, OC, device=dev, dtype=torch.bfloat16)
    stats = k.new_stats(OC, dev)
    sc = sh = None
    xe = x.float()
    if prologue:
        sc = torch.rand(IC, device=dev) + 0.5
        sh = torch.randn(IC, device=dev) * 0.1
        xe = torch.relu(x.float() * sc + sh).bfloat16().float()
    for tile in [None, (128, 128), (128, 64), (64, 64), (256, 128), (128, 256), (256, 64)]:
        if tile and OC % tile[1]:
            continue
        stats.zero_()
        k.conv_fwd(x, w.view(OC, -1), out, R=R, S=R, stride=st, pad=pad, stats=stats, in_scale=sc, in_shift=sh,
                   relu_in=True, tile=tile)
        ref = nhwc(F.conv2d(nchw(xe), w.float().permute(0, 3, 1, 2), stride=st, padding=pad))
        assert relerr(out, ref) < 1e-2, (tile, relerr(out, ref))
        s = stats.view(k.NSHARD, 2, OC).sum(0).float()
        o32 = out.float().view(-1, OC)
        assert relerr(s[0], o32.sum(0)) < 1e-3
        assert relerr(s[1], (o32 * o32).sum(0)) < 1e-3


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_dgrad(case):
    k = K()
    N, H, W, IC, OC, R, st, pad = case
    torch.manual_seed(1)
    w = (torch.randn(OC, R, R, IC, device=dev) / math.sqrt(IC * R * R)).bfloat16()
    OH, OW = k.conv_out_hw(H, W, R, R, st, pad)
    dy = torch.randn(N, OH, OW, OC, device=dev).bfloat16()
    wt = w.permute(3, 1, 2, 0).contiguous()  # [IC][R][S][OC]
    dx = torch.empty(N, H, W, IC, device=dev, dtype=torch.bfloat16)
    k.conv_dgrad(dy, wt.view(IC, -1), dx, R=R, S=R, stride=st, pad=pad)
    ref = torch.nn.grad.conv2d_input((N, IC, H, W), w.float().permute(0, 3, 1, 2), nchw(dy.float()),
                                     stride=st, padding=pad)
    assert relerr(dx, nhwc(ref)) < 1e-2
    # accumulate mode
    base = torch.randn_like(dx)
    dx2 = base.clone()
    k.conv_dgrad(dy, wt.view(IC, -1), dx2, R=R, S=R, stride=st, pad=pad, accumulate=True)
    assert relerr(dx2, nhwc(ref) + base.float()) < 1e-2


@pytest.mark.parametrize("case", CONV_CASES)
@pytest.mark.parametrize("prologue,dma", [(False, -1), (False, 0), (False, 2), (True, -1)])
def test_conv_wgrad(case, prologue, dma):
    k = K()
    N, H, W, IC, OC, R, st, pad = case
    torch.manual_seed(2)
    x = torch.randn(N, H, W, IC, device=dev).bfloat16()
    OH, OW = k.conv_out_hw(H, W, R, R, st, pad)
    dy = torch.randn(N, OH, OW, OC, device=dev).bfloat16()
    dw = torch.empty(OC, R * R * IC, device=dev)
    ws = torch.empty(64 * 1024 * 1024, device=dev)
    xe = x.float()
    sc = sh = None
    if prologue:
        sc = torch.rand(IC, device=dev) + 0.5
        sh = torch.randn(IC, device=dev) * 0.1
        xe = torch.relu(x.float() * sc + sh).bfloat16().float()
    ref = torch.nn.grad.conv2d_weight(nchw(xe), (OC, IC, R, R), nchw(dy.float()), stride=st, padding=pad)
    for tile in [None, (128, 128), (128, 64), (64, 128), (64, 64), (256, 128), (128, 256)]:
        if tile and (OC % tile[0] or IC % tile[1]):
            continue
        dw.fill_(float("nan"))
        k.conv_wgrad(dy, x, dw, ws, R=R, S=R, stride=st, pad=pad, in_scale=sc, in_shift=sh, tile=tile, dma=dma)
        assert relerr(dw.view(OC, R, R, IC), ref.permute(0, 2, 3, 1)) < 1e-2, tile


def test_stem_fwd_wgrad():
    k = K()
    N, H, W = 2, 32, 32
    torch.manual_seed(3)
    img = torch.randn(N, H, W, 3, device=dev)
    x4 = torch.zeros(N, H, W, 4, device=dev)
    x4[..., :3] = img
    x4 = x4.bfloat16()
    w = (torch.randn(64, 7, 7, 3, device=dev) * 0.05)
    ws_ = torch.zeros(64, 8, 8, 4, device=dev)
    ws_[:, :7, :7, :3] = w
    w16s = ws_.bfloat16().view(64, 256)
    OH, OW = k.conv_out_hw(H, W, 7, 7, 2, 3)
    out = torch.empty(N, OH, OW, 64, device=dev, dtype=torch.bfloat16)
    stats = k.new_stats(64, dev)
    k.conv_stem_fwd(x4, w16s, out, stats=stats)
    xr = nchw(x4[..., :3].float())
    wr = ws_.bfloat16().float()[:, :7, :7, :3].permute(0, 3, 1, 2)
    ref = nhwc(F.conv2d(xr, wr, stride=2, padding=3))
    assert relerr(out, ref) < 1e-2
    dy = torch.randn(N, OH, OW, 64, device=dev).bfloat16()
    dw = torch.empty(64, 256, device=dev)
    wsp = torch.empty(16 * 1024 * 1024, device=dev)
    k.conv_wgrad(dy, x4, dw, wsp, R=7, S=7, stride=2, pad=3, stem=True)
    refw = torch.nn.grad.conv2d_weight(xr, (64, 3, 7, 7), nchw(dy.float()), stride=2, padding=3)
    got = dw.view(64, 8, 8, 4)
    assert relerr(got[:, :7, :7, :3], refw.permute(0, 2, 3, 1)) < 1e-2
    assert got[:, 7].abs().max().item() == 0 and got[:, :, 7].abs().max().item() == 0


def _bn_ref_setup(M=4096, Cc=128):
    torch.manual_seed(4)
    y = (torch.randn(M, Cc, device=dev) * 2 + 0.5).bfloat16()
    return y


def test_bn_finalize_apply():
    k = K()
    M, Cc = 4096, 128
    y = _bn_ref_setup(M, Cc)
    stats = k.new_stats(Cc, dev)
    k.channel_stats(y, stats)
    gamma = torch.rand(Cc, device=dev) + 0.5
    beta = torch.randn(Cc, device=dev)
    rm = torch.zeros(Cc, device=dev)
    rv = torch.ones(Cc, device=dev)
    scale, shift, sm, si = (torch.empty(Cc, device=dev) for _ in range(4))
    k.bn_finalize(stats, M, gamma, beta, 1e-5, 0.1, rm, rv, scale, shift, sm, si)
    yf = y.float()
    mean = yf.mean(0)
    var = yf.var(0, unbiased=False)
    assert relerr(sm, mean) < 1e-4
    assert relerr(si, 1 / torch.sqrt(var + 1e-5)) < 1e-4
    assert relerr(rm, 0.1 * mean) < 1e-4
    assert relerr(rv, 0.9 + 0.1 * yf.var(0, unbiased=True)) < 1e-4
    out = torch.empty_like(y)
    res = torch.randn_like(yf).bfloat16()
    bits = torch.empty(y.numel() // 8, device=dev, dtype=torch.uint8)
    k.bn_apply(y, scale, shift, out, res=res, relu=True, mbits=bits)
    ref = torch.relu((yf - mean) / torch.sqrt(var + 1e-5) * gamma + beta + res.float())
    assert relerr(out, ref) < 1e-2
    assert torch.equal(bits, k.pack_mask_bits(out))  # 1-bit ReLU mask of the stored values
    assert torch.equal(k.unpack_mask_bits(bits, out.shape), out.float() > 0)
    rsc = torch.rand(Cc, device=dev)
    rsh = torch.randn(Cc, device=dev)
    k.bn_apply(y, scale, shift, out, res=res, res_scale=rsc, res_shift=rsh, relu=False)
    ref = (yf - mean) / torch.sqrt(var + 1e-5) * gamma + beta + res.float() * rsc + rsh
    assert relerr(out, ref) < 1e-2


@pytest.mark.parametrize("mask_mode", [0, 1, 2])
def test_bn_backward(mask_mode):
    k = K()
    M, Cc = 4096, 64
    y = _bn_ref_setup(M, Cc)
    gamma = torch.rand(Cc, device=dev) + 0.5
    beta = torch.randn(Cc, device=dev)
    yf = y.float().requires_grad_(True)
    bn = torch.nn.functional.batch_norm(yf, None, None, gamma, beta, training=True, eps=1e-5)
    dout = torch.randn(M, Cc, device=dev).bfloat16()
    mref = None
    if mask_mode == 0:
        target = bn
    elif mask_mode == 1:
        mref = torch.randn(M, Cc, device=dev).bfloat16()
        target = bn * (mref.float() > 0)
    else:
        target = torch.relu(bn)
    gam = gamma.clone().requires_grad_(True)
    bet = beta.clone().requires_grad_(True)
    yf2 = y.float().requires_grad_(True)
    bn2 = torch.nn.functional.batch_norm(yf2, None, None, gam, bet, training=True, eps=1e-5)
    if mask_mode == 1:
        t2 = bn2 * (mref.float() > 0)
    elif mask_mode == 2:
        t2 = torch.relu(bn2)
    else:
        t2 = bn2
    t2.backward(dout.float())
    mean = y.float().mean(0)
    invstd = 1 / torch.sqrt(y.float().var(0, unbiased=False) + 1e-5)
    scale = gamma * invstd
    shift = beta - mean * scale
    stats = k.new_stats(Cc, dev)
    k.bn_bwd_reduce(dout, y, mean, invstd, stats, mask_mode=mask_mode, mref=mref, scale=scale, shift=shift)
    coeff = torch.empty(3 * Cc, device=dev)
    dg = torch.empty(Cc, device=dev)
    db = torch.empty(Cc, device=dev)
    k.bn_bwd_coeff(stats, M, gamma, mean, invstd, coeff, dg, db)
    dy = torch.empty_like(y)
    gout = torch.empty_like(y)
    k.bn_bwd_apply(dout, y, coeff, dy, mask_mode=mask_mode, mref=mref, scale=scale, shift=shift, gout=gout)
    assert relerr(dy, yf2.grad) < 2e-2
    assert relerr(dg, gam.grad) < 1e-3
    assert relerr(db, bet.grad) < 1e-3


def test_maxpool():
    k = K()
    N, H, W, Cc = 2, 16, 16, 64
    torch.manual_seed(5)
    x = torch.randn(N, H, W, Cc, device=dev).bfloat16()
    sc = torch.rand(Cc, device=dev) + 0.5
    sh = torch.randn(Cc, device=dev) * 0.1
    out = torch.empty(N, 8, 8, Cc, device=dev, dtype=torch.bfloat16)
    arg = torch.empty(N, 8, 8, Cc, device=dev, dtype=torch.uint8)
    k.maxpool_fwd(x, out, arg, scale=sc, shift=sh, relu=True)
    act = torch.relu(x.float() * sc + sh).requires_grad_(True)
    ref = F.max_pool2d(nchw(act), 3, 2, 1)
    assert relerr(out, nhwc(ref)) < 1e-2
    dout = torch.randn(N, 8, 8, Cc, device=dev).bfloat16()
    ref.backward(nchw(dout.float()))
    dx = torch.empty_like(x)
    k.maxpool_bwd(dout, arg, dx)
    # ties (relu zeros) may route differently; compare on positive activations only
    m = (act.detach() > 0)
    assert relerr(dx.float() * m, act.grad * m) < 2e-2


def test_maxpool_ymax_matches_reference_and_stem_reduce():
    """maxpool_fwd's ymax (raw input at the argmax) equals the reference's, and the stem BN-backward
    reduction over pooled positions (dpool, ymax, MASK_Y) equals the full-resolution gather form."""
    k = K()
    from dbx_distributed_pytorch_examples_amd.ops import reference as R
    N, H, W, Cc = 2, 112, 112, 64
    torch.manual_seed(6)
    x = torch.randn(N, H, W, Cc, device=dev).bfloat16()
    sc, sh = torch.rand(Cc, device=dev) + 0.5, torch.randn(Cc, device=dev) * 0.1
    out, arg, ym = (torch.empty(N, 56, 56, Cc, device=dev, dtype=t) for t in (torch.bfloat16, torch.uint8,
                                                                               torch.bfloat16))
    k.maxpool_fwd(x, out, arg, scale=sc, shift=sh, relu=True, ymax=ym)
    xc, oc, ac, yc = x.cpu(), torch.empty_like(out).cpu(), torch.empty_like(arg).cpu(), torch.empty_like(ym).cpu()
    R.maxpool_fwd(xc, oc, ac, scale=sc.cpu(), shift=sh.cpu(), relu=True, ymax=yc)
    assert torch.equal(out.cpu(), oc) and torch.equal(arg.cpu(), ac) and torch.equal(ym.cpu(), yc)
    dp = torch.randn(N, 56, 56, Cc, device=dev).bfloat16()
    mean, inv = torch.randn(Cc, device=dev) * 0.1, torch.rand(Cc, device=dev) + 0.5
    st_full, st_pool = k.new_stats(Cc, dev), k.new_stats(Cc, dev)
    k.pool_bn_bwd_reduce(dp, arg, x, sc, sh, mean, inv, st_full, K=3, stride=2, pad=1)
    k.bn_bwd_reduce(dp, ym, mean, inv, st_pool, mask_mode=k.MASK_Y, scale=sc, shift=sh)
    a, b = st_full.view(-1, 2, Cc).sum(0), st_pool.view(-1, 2, Cc).sum(0)
    assert ((a - b).abs() / (a.abs() + 1.0)).max().item() < 1e-4


@pytest.mark.parametrize("hw", [(16, 16), (15, 13), (112, 112)])
def test_pool_bn_bwd_fused(hw):
    """Stem backward with the max-pool backward folded into the BN reduce/apply passes, against
    fp32 autograd of relu(bn(y)) -> maxpool (odd sizes exercise the window-edge cases)."""
    k = K()
    H, W = hw
    N, Cc = (2 if H > 64 else 3), 64
    torch.manual_seed(6)
    y = torch.randn(N, H, W, Cc, device=dev).bfloat16()
    mean = y.float().mean((0, 1, 2))
    invstd = 1.0 / y.float().var((0, 1, 2), unbiased=False).add(1e-5).sqrt()
    gamma = torch.rand(Cc, device=dev) + 0.5
    beta = torch.randn(Cc, device=dev) * 0.2
    sc, sh = (gamma * invstd).contiguous(), (beta - mean * gamma * invstd).contiguous()
    P, Q = (H + 2 - 3) // 2 + 1, (W + 2 - 3) // 2 + 1
    pooled = torch.empty(N, P, Q, Cc, device=dev, dtype=torch.bfloat16)
    arg = torch.empty(N, P, Q, Cc, device=dev, dtype=torch.uint8)
    k.maxpool_fwd(y, pooled, arg, scale=sc, shift=sh, relu=True)
    dpool = torch.randn(N, P, Q, Cc, device=dev).bfloat16()
    # fp32 reference: BN (batch stats) -> relu -> maxpool, autograd
    yr = y.float().requires_grad_(True)
    xh = (yr - mean) * invstd
    out = F.max_pool2d(nchw(torch.relu(xh * gamma + beta)), 3, 2, 1)
    out.backward(nchw(dpool.float()))
    # the batch-statistics BN backward of the same graph: dy = gamma*invstd*(g - mean(g) - xhat*mean(g*xhat))
    act = torch.relu(xh * gamma + beta).detach().requires_grad_(True)
    F.max_pool2d(nchw(act), 3, 2, 1).backward(nchw(dpool.float()))
    g = act.grad * (act.detach() > 0)
    xhd = xh.detach()
    cnt = N * H * W
    sg, sgx = g.sum((0, 1, 2)), (g * xhd).sum((0, 1, 2))
    dy_ref = gamma * invstd * (g - sg / cnt - xhd * sgx / cnt)
    stats = k.new_stats(Cc, dev)
    k.pool_bn_bwd_reduce(dpool, arg, y, sc, sh, mean.contiguous(), invstd.contiguous(), stats)
    st = stats.view(k.NSHARD, 2, Cc).sum(0)
    assert relerr(st[0], sg) < 1e-3 and relerr(st[1], sgx) < 1e-3
    coeff = torch.empty(3 * Cc, device=dev)
    dgamma, dbeta = torch.empty(Cc, device=dev), torch.empty(Cc, device=dev)
    k.bn_bwd_coeff(stats, cnt, gamma, mean.contiguous(), invstd.contiguous(), coeff, dgamma, dbeta)
    dy = torch.empty_like(y)
    k.pool_bn_bwd_apply(dpool, arg, y, sc, sh, coeff, dy)
    assert relerr(dy, dy_ref) < 2e-2
    assert relerr(dbeta, sg) < 1e-3 and relerr(dgamma, sgx) < 1e-3
    # CPU reference implementation agrees with the kernel
    st_ref = k.new_stats(Cc, "cpu")
    cpu = lambda t: t.cpu()  # noqa: E731
    from dbx_distributed_pytorch_examples_amd.ops import reference as R
    R.pool_bn_bwd_reduce(cpu(dpool), cpu(arg), cpu(y), cpu(sc), cpu(sh), cpu(mean), cpu(invstd), st_ref)
    assert relerr(st_ref.view(k.NSHARD, 2, Cc).sum(0), st.cpu()) < 1e-4


def test_avgpool():
    k = K()
    x = torch.randn(4, 7, 7, 256, device=dev).bfloat16()
    out = torch.empty(4, 256, device=dev, dtype=torch.bfloat16)
    k.avgpool_fwd(x, out)
    assert relerr(out, x.float().mean((1, 2))) < 1e-2
    d = torch.randn(4, 256, device=dev).bfloat16()
    dx = torch.empty_like(x)
    k.avgpool_bwd(d, dx)
    assert relerr(dx, (d.float() / 49)[:, None, None, :].expand(4, 7, 7, 256)) < 1e-2


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("smoothing", [0.0, 0.1])
def test_softmax_ce(dtype, smoothing):
    k = K()
    B, Cc = 64, 1000
    torch.manual_seed(6)
    logits = (torch.randn(B, Cc, device=dev) * 3).to(dtype)
    labels = torch.randint(0, Cc, (B,), device=dev)
    lf = logits.float().requires_grad_(True)
    loss = F.cross_entropy(lf, labels, label_smoothing=smoothing)
    loss.backward()
    dl = torch.empty_like(logits)
    lo = torch.empty(B, device=dev)
    st = torch.zeros(2, device=dev, dtype=torch.float64)
    k.softmax_ce(logits, labels, dl, lo, st, smoothing=smoothing)
    assert abs(lo.mean().item() - loss.item()) < 1e-3 * max(1, loss.item())
    assert abs(st[0].item() / B - loss.item()) < 1e-3 * max(1, loss.item())
    assert st[1].item() == (logits.float().argmax(1) == labels).sum().item()
    assert relerr(dl, lf.grad) < 1e-2


def test_sgd_adam():
    k = K()
    n = 100003
    torch.manual_seed(7)
    p = torch.randn(n, device=dev)
    g = torch.randn(n, device=dev)
    ref = torch.nn.Parameter(p.clone())
    opt = torch.optim.SGD([ref], lr=0.1, momentum=0.9, weight_decay=1e-4, nesterov=True)
    v = torch.zeros(n, device=dev)
    p16 = torch.empty(n, device=dev, dtype=torch.bfloat16)
    for step in range(3):
        ref.grad = g.clone()
        opt.step()
        k.sgd_step(p, g, v, p16, lr=0.1, momentum=0.9, weight_decay=1e-4, nesterov=True, first=(step == 0))
    assert relerr(p, ref.detach()) < 1e-5
    assert relerr(p16, ref.detach()) < 1e-2
    p = torch.randn(n, device=dev)
    ref = torch.nn.Parameter(p.clone())
    opt = torch.optim.AdamW([ref], lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01)
    m = torch.zeros(n, device=dev)
    v = torch.zeros(n, device=dev)
    for step in range(1, 4):
        ref.grad = g.clone()
        opt.step()
        k.adam_step(p, g, m, v, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.01, decoupled=True,
                    step=step)
    assert relerr(p, ref.detach()) < 1e-5


def test_clip_factor():
    k = K()
    g = torch.randn(1 << 20, device=dev)
    work = torch.zeros(4, device=dev)
    f = k.global_norm_clip_factor(g, 1.0, work)
    nrm = g.norm().item()
    assert abs(work[3].item() - nrm) / nrm < 1e-4
    assert abs(f.item() - min(1.0, 1.0 / (nrm + 1e-6))) < 1e-6


def test_normalize_u8():
    k = K()
    img = torch.randint(0, 256, (3, 8, 8, 3), device=dev, dtype=torch.uint8)
    out = torch.empty(3, 8, 8, 4, device=dev, dtype=torch.bfloat16)
    mean, std = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)
    flip = torch.tensor([0, 1, 0], device=dev, dtype=torch.uint8)
    k.normalize_u8(img, out, mean, std, flip)
    ref = (img.float() / 255 - torch.tensor(mean, device=dev)) / torch.tensor(std, device=dev)
    ref[1] = ref[1].flip(1)
    assert relerr(out[..., :3], ref) < 1e-2
    assert out[..., 3].abs().max().item() == 0


@pytest.mark.parametrize("shape", [(16, 56, 56, 64, 64, 1, 1, 0), (8, 28, 28, 128, 128, 3, 1, 1),
                                   (8, 28, 28, 256, 512, 1, 2, 0)])
def test_conv_wgrad_split(shape):
    """Large pixel counts -> many split-K slabs and the 2-level reduction."""
    k = K()
    N, H, W, IC, OC, R, st, pad = shape
    torch.manual_seed(8)
    x = torch.randn(N, H, W, IC, device=dev).bfloat16()
    OH, OW = k.conv_out_hw(H, W, R, R, st, pad)
    dy = torch.randn(N, OH, OW, OC, device=dev).bfloat16()
    dw = torch.empty(OC, R * R * IC, device=dev)
    ws = torch.empty(64 * 1024 * 1024, device=dev)
    nsplit, _ = k.wgrad_splits(N * OH * OW, OC, R * R * IC, 64, 64, ws.numel())
    assert nsplit > 1
    ref = torch.nn.grad.conv2d_weight(nchw(x.float()), (OC, IC, R, R), nchw(dy.float()), stride=st, padding=pad)
    for tile in [None, (256, 128), (128, 256)]:
        if tile and (OC % tile[0] or IC % tile[1]):
            continue
        for dma in (3, 2, 0):  # LDS-DMA rings of depth 3 / 2, register-staged
            dw.fill_(float("nan"))
            k.conv_wgrad(dy, x, dw, ws, R=R, S=R, stride=st, pad=pad, tile=tile, dma=dma)
            assert relerr(dw.view(OC, R, R, IC), ref.permute(0, 2, 3, 1)) < 1e-2, (tile, dma)


@pytest.mark.parametrize("shape", [(8, 28, 28, 256, 512, 1, 2, 0), (4, 14, 14, 256, 256, 3, 1, 1),
                                   (16, 14, 14, 256, 1024, 1, 1, 0), (8, 7, 7, 512, 512, 3, 1, 1)])
@pytest.mark.parametrize("dma", [4, 2])
@pytest.mark.parametrize("rounds", [0.0, 1.0, 4.0])
def test_conv_wgrad_256x256(shape, dma, rounds):
    """The 256 x 256 weight-gradient tile (2 x 4 waves of 128 x 64; dma 4: 32-pixel stages in a
    4-slot LDS-DMA ring, dma 2: 64-pixel stages in 2 slots) against fp32, unsplit (written straight
    to dW), split with the separate reduce, and split with the in-launch reduction (tile counters)."""
    k = K()
    N, H, W, IC, OC, R, st, pad = shape
    torch.manual_seed(9)
    x = torch.randn(N, H, W, IC, device=dev).bfloat16()
    OH, OW = k.conv_out_hw(H, W, R, R, st, pad)
    dy = torch.randn(N, OH, OW, OC, device=dev).bfloat16()
    dw = torch.empty(OC, R * R * IC, device=dev)
    ws = torch.empty(64 * 1024 * 1024, device=dev)
    ref = torch.nn.grad.conv2d_weight(nchw(x.float()), (OC, IC, R, R), nchw(dy.float()), stride=st, padding=pad)
    for cnt in (None, torch.zeros(k.wgrad_tiles_max(OC, R * R * IC), dtype=torch.int32, device=dev)):
        dw.fill_(float("nan"))
        k.conv_wgrad(dy, x, dw, ws, R=R, S=R, stride=st, pad=pad, tile=(256, 256), dma=dma, rounds=rounds, cnt=cnt)
        assert relerr(dw.view(OC, R, R, IC), ref.permute(0, 2, 3, 1)) < 1e-2, (dma, rounds, cnt is not None)
        if cnt is not None:
            assert int(cnt.abs().sum()) == 0  # counters reset for the next launch


def test_stem_wgrad_split():
    k = K()
    N, H, W = 8, 64, 64
    torch.manual_seed(9)
    x4 = torch.zeros(N, H, W, 4, device=dev)
    x4[..., :3] = torch.randn(N, H, W, 3, device=dev)
    x4 = x4.bfloat16()
    dy = torch.randn(N, 32, 32, 64, device=dev).bfloat16()
    dw = torch.empty(64, 256, device=dev)
    wsp = torch.empty(16 * 1024 * 1024, device=dev)
    k.conv_wgrad(dy, x4, dw, wsp, R=7, S=7, stride=2, pad=3, stem=True)
    refw = torch.nn.grad.conv2d_weight(nchw(x4[..., :3].float()), (64, 3, 7, 7), nchw(dy.float()), stride=2, padding=3)
    assert relerr(dw.view(64, 8, 8, 4)[:, :7, :7, :3], refw.permute(0, 2, 3, 1)) < 1e-2


def test_conv_dgrad_stride2_tiles():
    """Parity-decomposed stride-2 dgrad on every tile config."""
    k = K()
    N, H, W, IC, OC, R, st, pad = 4, 14, 14, 128, 256, 3, 2, 1
    w = (torch.randn(OC, R, R, IC, device=dev) / math.sqrt(IC * R * R)).bfloat16()
    dy = torch.randn(N, 7, 7, OC, device=dev).bfloat16()
    wt = w.permute(3, 1, 2, 0).contiguous().view(IC, -1)
    ref = nhwc(torch.nn.grad.conv2d_input((N, IC, H, W), w.float().permute(0, 3, 1, 2), nchw(dy.float()),
                                          stride=st, padding=pad))
    for tile in [(128, 128), (128, 64), (64, 64), (256, 128), (128, 256), (256, 64)]:
        if IC % tile[1]:
            continue
        dx = torch.full((N, H, W, IC), 7.0, device=dev, dtype=torch.bfloat16)
        k.conv_dgrad(dy, wt, dx, R=R, S=R, stride=st, pad=pad, tile=tile)
        assert relerr(dx, ref) < 1e-2, tile


def test_augment_u8_matches_reference():
    k = K()
    from dbx_distributed_pytorch_examples_amd.ops import reference as R
    torch.manual_seed(10)
    img = torch.randint(0, 256, (4, 40, 36, 3), device=dev, dtype=torch.uint8)
    boxes = torch.tensor([[0, 0, 40, 36], [3.0, 2.0, 20.0, 30.0], [-4, -4, 32, 32], [10, 5, 12, 12]], device=dev)
    flip = torch.tensor([0, 1, 0, 1], device=dev, dtype=torch.uint8)
    out = torch.empty(4, 32, 32, 4, device=dev, dtype=torch.bfloat16)
    mean, std = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)
    k.augment_u8(img, out, boxes, mean, std, flip)
    ref_cpu = torch.empty(4, 32, 32, 4, dtype=torch.bfloat16)
    R.augment_u8(img.cpu(), ref_cpu, boxes.cpu(), mean, std, flip.cpu())
    assert relerr(out.cpu(), ref_cpu) < 1e-2


@pytest.mark.parametrize("mode,sub,stride", [(1, 1, 1), (1, 2, 1), (2, 1, 1), (2, 1, 2), (0, 2, 1)])
def test_conv_dgrad_fused_epilogue(mode, sub, stride):
    """dgrad + residual addend (sub-sampled) + BN-backward epilogue vs the reference semantics."""
    k = K()
    from dbx_distributed_pytorch_examples_amd.ops import reference as R
    torch.manual_seed(11)
    N, H, W, IC, OC, Rr = 2, 8, 8, 256, 128, 3
    pad = 1
    P = (H + 2 * pad - Rr) // stride + 1
    w = (torch.randn(OC, Rr, Rr, IC, device=dev) / math.sqrt(IC * 9)).bfloat16()
    wt = w.permute(3, 1, 2, 0).contiguous().view(IC, -1)
    dy = torch.randn(N, P, P, OC, device=dev).bfloat16()
    add = torch.randn(N, H // sub, W // sub, IC, device=dev).bfloat16()
    ybn = torch.randn(N, H, W, IC, device=dev).bfloat16()
    ybn2 = torch.randn(N, H, W, IC, device=dev).bfloat16()
    mref = torch.randn(N, H, W, IC, device=dev).bfloat16()
    mean, inv = torch.randn(IC, device=dev) * 0.1, torch.rand(IC, device=dev) + 0.5
    mean2, inv2 = torch.randn(IC, device=dev) * 0.1, torch.rand(IC, device=dev) + 0.5
    sc, sh = torch.rand(IC, device=dev) + 0.5, torch.randn(IC, device=dev) * 0.1

    def run(mod, devc, tile=None):
        t = lambda v: v.to(devc)  # noqa: E731
        st1 = k.new_stats(IC, devc)
        st2 = k.new_stats(IC, devc)
        epi = None
        if mode:
            epi = k.BNBwdEpilogue(mode, t(ybn), t(mean), t(inv), st1,
                                  mbits=k.pack_mask_bits(t(mref)) if mode == 1 else None,
                                  scale=t(sc) if mode == 2 else None, shift=t(sh) if mode == 2 else None,
                                  ybn2=t(ybn2) if mode == 1 else None, mean2=t(mean2), inv2=t(inv2),
                                  stats2=st2 if mode == 1 else None)
        dx = torch.empty(N, H, W, IC, device=devc, dtype=torch.bfloat16)
        mod.conv_dgrad(t(dy), t(wt), dx, R=Rr, S=Rr, stride=stride, pad=pad, addsrc=t(add), add_sub=sub, epilogue=epi,
                       tile=tile)
        return dx.float().cpu(), st1.view(k.NSHARD, 2, IC).sum(0).float().cpu(), st2.view(k.NSHARD, 2, IC).sum(0).float().cpu()

    r_dx, r_s1, r_s2 = run(R, "cpu")
    for tile in [None, (128, 128), (64, 64), (256, 128), (128, 256), (256, 64)]:
        g_dx, g_s1, g_s2 = run(k, dev, tile)
        assert relerr(g_dx, r_dx) < 2e-2, tile
        if mode:
            assert relerr(g_s1, r_s1) < 2e-2, tile
            if mode == 1:
                assert relerr(g_s2, r_s2) < 2e-2, tile


def test_bn_bwd_apply2_matches_two_applies():
    k = K()
    torch.manual_seed(11)
    N, H, W, Cc = 3, 7, 5, 128
    g = torch.randn(N, H, W, Cc, device=dev).bfloat16()
    y1, y2 = torch.randn_like(g), torch.randn_like(g)
    c1, c2 = torch.randn(3 * Cc, device=dev), torch.randn(3 * Cc, device=dev)
    d1, d2 = torch.empty_like(g), torch.empty_like(g)
    k.bn_bwd_apply2(g, y1, c1, d1, y2, c2, d2)
    for y, c, d in ((y1, c1, d1), (y2, c2, d2)):
        kk = c.view(3, Cc)
        ref = kk[0] * g.float() + kk[1] * y.float() + kk[2]
        assert relerr(d, ref) < 1e-2


@pytest.mark.parametrize("case", [(2, 14, 14, 64, 64, 3, 1, 1), (2, 14, 14, 128, 256, 1, 1, 0), (3, 7, 7, 512, 512, 3, 1, 1),
                                  (4, 9, 9, 64, 128, 3, 2, 1), (2, 14, 14, 128, 128, 3, 2, 1)])
def test_dgrad_epilogue_act_out(case):
    """The MASK_Y dgrad epilogue also stores the BN output relu(ybn*scale+shift) (every element,
    strided phases included); gradient and statistics are unchanged by it."""
    k = K()
    N, H, W, IC, OC, R, st, pad = case
    torch.manual_seed(12)
    OH, OW = k.conv_out_hw(H, W, R, R, st, pad)
    w = (torch.randn(OC, R, R, IC, device=dev) / math.sqrt(IC * R * R)).bfloat16()
    wt = w.permute(3, 1, 2, 0).contiguous().view(IC, -1)
    dy = torch.randn(N, OH, OW, OC, device=dev).bfloat16()
    ybn = torch.randn(N, H, W, IC, device=dev).bfloat16()
    sc = torch.rand(IC, device=dev) + 0.5
    sh = torch.randn(IC, device=dev) * 0.1
    mean, inv = torch.randn(IC, device=dev) * 0.1, torch.rand(IC, device=dev) + 0.5
    act_ref = torch.relu(ybn.float() * sc + sh)
    outs = []
    for act in (None, torch.full_like(ybn, float("nan"))):
        st1 = k.new_stats(IC, dev)
        dx = torch.empty_like(ybn)
        e = k.BNBwdEpilogue(k.MASK_Y, ybn, mean, inv, st1, scale=sc, shift=sh, act_out=act)
        k.conv_dgrad(dy, wt, dx, R=R, S=R, stride=st, pad=pad, epilogue=e)
        outs.append((dx, st1))
        if act is not None:
            assert not torch.isnan(act.float()).any()
            assert relerr(act, act_ref) < 1e-2 and (act.float() - act_ref).abs().max().item() < 0.07
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("tile", [(64, 64), (128, 64), (128, 128), (256, 64), (256, 128), (128, 256)])
@pytest.mark.parametrize("case", [(2, 14, 14, 256, 64, False), (2, 7, 7, 1024, 256, True), (3, 9, 9, 512, 128, False)])
def test_conv_fwd_tail_prologue(case, tile):
    """conv1 with the tail prologue == bn_apply(conv3 out, shortcut) followed by a plain conv1: the
    block output and its ReLU mask are written back as bn_apply writes them, the conv output and the
    BN statistics match (identity shortcut: bit-exact block output)."""
    k = K()
    N, H, W, IC, OC, ds = case
    if OC % tile[1]:
        pytest.skip("tile wider than OC")
    torch.manual_seed(21)
    x = torch.randn(N, H, W, IC, device=dev).bfloat16()
    res = torch.randn(N, H, W, IC, device=dev).bfloat16()
    sc, sh = torch.rand(IC, device=dev) + 0.5, torch.randn(IC, device=dev) * 0.1
    rsc, rsh = (torch.rand(IC, device=dev) + 0.5, torch.randn(IC, device=dev) * 0.1) if ds else (None, None)
    w = (torch.randn(OC, 1, 1, IC, device=dev) / math.sqrt(IC)).bfloat16()
    out_ref, bits_ref = torch.empty_like(x), torch.empty(x.numel() // 8, device=dev, dtype=torch.uint8)
    k.bn_apply(x, sc, sh, out_ref, res=res, res_scale=rsc, res_shift=rsh, relu=True, mbits=bits_ref)
    y_ref, st_ref = torch.empty(N, H, W, OC, device=dev).bfloat16(), k.new_stats(OC, dev)
    k.conv_fwd(out_ref, w, y_ref, R=1, S=1, stride=1, pad=0, stats=st_ref, tile=tile)
    out, bits = torch.full_like(x, float("nan")), torch.zeros_like(bits_ref)
    y, st = torch.empty_like(y_ref), k.new_stats(OC, dev)
    k.conv_fwd(x, w, y, R=1, S=1, stride=1, pad=0, stats=st, in_scale=sc, in_shift=sh, tile=tile, tail_res=res,
               tail_res_scale=rsc, tail_res_shift=rsh, tail_out=out, tail_bits=bits)
    torch.cuda.synchronize()
    if ds:
        assert (out.float() - out_ref.float()).abs().max().item() < 0.07
        assert (bits != bits_ref).float().mean().item() < 1e-3
        assert relerr(y, y_ref) < 1e-2
    else:
        assert torch.equal(out, out_ref) and torch.equal(bits, bits_ref)
        assert relerr(y, y_ref) < 2e-3
    s, s_ref = st.view(-1, 2, OC).sum(0), st_ref.view(-1, 2, OC).sum(0)
    assert ((s - s_ref).abs() / (s_ref.abs() + N * H * W)).max().item() < 1e-2


@pytest.mark.parametrize("tile", [(64, 64), (128, 64), (128, 128), (256, 64), (256, 128), (128, 256)])
@pytest.mark.parametrize("variant", ["epi2", "epi1_acc", "acc", "plain"])
@pytest.mark.parametrize("cc", [128, 256])
def test_dgrad_bwd_apply_prologue(variant, tile, cc):
    """1x1 dgrad whose operand is the BN-backward apply k1*g + k2*y + k3 computed while staging ==
    bn_bwd_apply followed by the plain dgrad (same epilogue); the applied operand is stored.
    (cc 256: the 128 x 256 tile covers every output channel in one N tile)"""
    k = K()
    N, H, W, Kc, Cc = 2, 14, 14, 256, cc
    if Cc % tile[1]:
        pytest.skip("tile wider than C")
    torch.manual_seed(31)
    g = torch.randn(N, H, W, Kc, device=dev).bfloat16()
    y = torch.randn(N, H, W, Kc, device=dev).bfloat16()
    coeff = torch.randn(3 * Kc, device=dev) * 0.5
    wt = (torch.randn(Cc, Kc, device=dev) / math.sqrt(Kc)).bfloat16()
    ybn = torch.randn(N, H, W, Cc, device=dev).bfloat16()
    mean, inv = torch.randn(Cc, device=dev) * 0.1, torch.rand(Cc, device=dev) + 0.5
    sc, sh = torch.rand(Cc, device=dev) + 0.5, torch.randn(Cc, device=dev) * 0.1
    add = torch.randn(N, H, W, Cc, device=dev).bfloat16()
    mbits = k.pack_mask_bits(torch.randn(N, H, W, Cc, device=dev).bfloat16())

    def run(dy_in, **kw):
        st1 = k.new_stats(Cc, dev)
        dx = torch.empty(N, H, W, Cc, device=dev, dtype=torch.bfloat16)
        if variant == "epi2":
            e = k.BNBwdEpilogue(k.MASK_Y, ybn, mean, inv, st1, scale=sc, shift=sh)
            k.conv_dgrad(dy_in, wt, dx, R=1, S=1, stride=1, pad=0, tile=tile, epilogue=e, **kw)
        elif variant == "epi1_acc":
            e = k.BNBwdEpilogue(k.MASK_OUT, ybn, mean, inv, st1, mbits=mbits)
            k.conv_dgrad(dy_in, wt, dx, R=1, S=1, stride=1, pad=0, tile=tile, epilogue=e, addsrc=add, **kw)
        elif variant == "acc":
            k.conv_dgrad(dy_in, wt, dx, R=1, S=1, stride=1, pad=0, tile=tile, addsrc=add, **kw)
        else:
            k.conv_dgrad(dy_in, wt, dx, R=1, S=1, stride=1, pad=0, tile=tile, **kw)
        return dx, st1

    dy_ref = torch.empty_like(g)
    k.bn_bwd_apply(g, y, coeff, dy_ref, mask_mode=k.MASK_NONE)
    dx_ref, st_ref = run(dy_ref)
    dy_out = torch.full_like(g, float("nan"))
    dx, st = run(g, bwd_y=y, bwd_coeff=coeff, dy_out=dy_out)
    torch.cuda.synchronize()
    assert (dy_out.float() - dy_ref.float()).abs().max().item() <= 0.02 * dy_ref.float().abs().max().item()
    assert relerr(dx, dx_ref) < 1e-2
    if variant in ("epi2", "epi1_acc"):
        a, b = st.view(-1, 2, Cc).sum(0), st_ref.view(-1, 2, Cc).sum(0)
        assert ((a - b).abs() / (b.abs() + N * H * W * 0.01)).max().item() < 2e-2


@pytest.mark.parametrize("dma", [0, 1])
@pytest.mark.parametrize("tile", [(128, 128), (128, 256), (256, 128), (128, 64), (64, 64)])
@pytest.mark.parametrize("R", [1, 3])
def test_conv_fwd_persistent_many_tiles(tile, R, dma):
    """Far more tiles than resident workgroups (each workgroup walks several tiles, staging the
    next tile's first block during the epilogue; dma 1: weights by LDS-DMA, DMA-ed after the
    epilogue): output and BN statistics vs fp32 torch."""
    tile = tuple(tile) + (dma,)
    k = K()
    N, H, W, IC, OC = 24, 56, 56, 64, 256
    torch.manual_seed(41)
    x = torch.randn(N, H, W, IC, device=dev).bfloat16()
    sc, sh = torch.rand(IC, device=dev) + 0.5, torch.randn(IC, device=dev) * 0.1
    w = (torch.randn(OC, R, R, IC, device=dev) / math.sqrt(IC * R * R)).bfloat16()
    y = torch.empty(N, H, W, OC, device=dev, dtype=torch.bfloat16)
    st = k.new_stats(OC, dev)
    k.conv_fwd(x, w.view(OC, -1), y, R=R, S=R, stride=1, pad=R // 2, stats=st, in_scale=sc, in_shift=sh, tile=tile)
    act = torch.relu(x.float() * sc + sh).bfloat16().float()
    ref = F.conv2d(nchw(act), w.float().permute(0, 3, 1, 2), padding=R // 2)
    assert relerr(y, nhwc(ref)) < 1e-2
    s = st.view(-1, 2, OC).sum(0)
    yf = y.float().view(-1, OC)
    assert ((s[0] - yf.sum(0)).abs() / (yf.abs().sum(0) + 1)).max().item() < 1e-3
    assert ((s[1] - (yf * yf).sum(0)).abs() / ((yf * yf).sum(0) + 1)).max().item() < 1e-3
