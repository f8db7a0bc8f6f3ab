"""PyTorch reference implementations of every HIP kernel, with identical signatures.

``ops.kernels`` dispatches here for CPU tensors, which makes the whole native program
(``engine.program``) runnable — and testable, including the DDP bucket path over gloo — on a
host without a GPU. They are the semantic definition the HIP kernels are tested against
(tests/test_kernels_gpu.py compares the kernels to plain fp32 torch ops of the same math).
Numerics mirror the kernels: bf16 storage, fp32 accumulation, prologue output rounded to bf16.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

NSHARD = 32  # BN-statistics shards of the large steps (see kernels.NSHARD; small steps use 4: EngineConfig.nshard)
MASK_NONE, MASK_OUT, MASK_Y = 0, 1, 2


def _nchw(x):
    return x.permute(0, 3, 1, 2)


def _nhwc(x):
    return x.permute(0, 2, 3, 1)


def _act_in(x, in_scale, in_shift, relu_in):
    xf = x.float()
    if in_scale is not None:
        xf = xf * in_scale + in_shift
        if relu_in:
            xf = torch.relu(xf)
        xf = xf.bfloat16().float()
    return xf


def _add_stats(stats, y):
    C = y.shape[-1]
    yf = y.float().reshape(-1, C)
    st = stats.view(-1, 2, C)
    st[0, 0] += yf.sum(0)
    st[0, 1] += (yf * yf).sum(0)


def conv_fwd(x, w16, out, *, R, S, stride, pad, stats=None, in_scale=None, in_shift=None, relu_in=True, tile=None,
             tail_res=None, tail_res_scale=None, tail_res_shift=None, tail_out=None, tail_bits=None, fin=None,
             fin_in=None, fin_in_res=None):
    for f in (fin_in, fin_in_res):  # the input BNs' finalizes, done by the consumer on the GPU
        if f is not None:
            f.run()
    OC = w16.shape[0]
    IC = x.shape[-1]
    if tail_res is not None:  # previous block's output relu(bn3(x) + shortcut): bn_apply's semantics
        act = tail_out if tail_out is not None else torch.empty_like(x)
        bn_apply(x, in_scale, in_shift, act, res=tail_res, res_scale=tail_res_scale, res_shift=tail_res_shift,
                 relu=True, mbits=tail_bits)
        xf = act.float()
    else:
        xf = _act_in(x, in_scale, in_shift, relu_in)
    w = w16.float().view(OC, R, S, IC).permute(0, 3, 1, 2)
    y = _nhwc(F.conv2d(_nchw(xf), w, stride=stride, padding=pad)).bfloat16()
    out.copy_(y.reshape(out.shape))
    if stats is not None:
        _add_stats(stats, out)
        if fin is not None:  # the kernels' in-launch BN finalize, as its own step
            fin.run()
    return out


def conv_dgrad(dy, wt16, dx, *, R, S, stride, pad, accumulate=False, tile=None, addsrc=None, add_sub=1,
               epilogue=None, bwd_y=None, bwd_coeff=None, dy_out=None, _fin=(0, 1)):
    if bwd_y is not None:  # the operand is the BN-backward apply of (dy, bwd_y)
        d = dy_out if dy_out is not None else torch.empty_like(dy)
        bn_bwd_apply(dy, bwd_y, bwd_coeff, d, mask_mode=MASK_NONE)
        dy = d
    N, P, Q, Kc = dy.shape
    _, H, W, Cc = dx.shape
    w = wt16.float().view(Cc, R, S, Kc).permute(3, 0, 1, 2)  # [K, C, R, S]
    g = torch.nn.grad.conv2d_input((N, Cc, H, W), w, _nchw(dy.float()), stride=stride, padding=pad)
    g = _nhwc(g).bfloat16().float()  # the kernel rounds the tile to bf16 before the epilogue
    if addsrc is not None:
        add = torch.zeros_like(g)
        add[:, ::add_sub, ::add_sub] = addsrc.float()
        g = g + add
    elif accumulate:
        g = g + dx.float()
    if epilogue is not None:
        e = epilogue
        y = e.ybn.float()
        if e.mode == MASK_OUT:
            w = 2 ** torch.arange(8, dtype=torch.int32, device=g.device)
            bits = (e.mbits.to(torch.int32).view(-1, 1) & w) != 0
            g = g * bits.reshape(g.shape)
        else:
            t = y * e.scale + e.shift
            g = g * (t > 0)
            if getattr(e, "act_out", None) is not None:
                e.act_out.copy_(torch.relu(t).bfloat16())
        g = g.bfloat16().float()
        gf = g.reshape(-1, Cc)
        st = e.stats1.view(-1, 2, Cc)
        st[0, 0] += gf.sum(0)
        st[0, 1] += (gf * ((y - e.mean1) * e.inv1).reshape(-1, Cc)).sum(0)
        if e.ybn2 is not None:
            st2 = e.stats2.view(-1, 2, Cc)
            st2[0, 0] += gf.sum(0)
            st2[0, 1] += (gf * ((e.ybn2.float() - e.mean2) * e.inv2).reshape(-1, Cc)).sum(0)
        if hasattr(e, "run_fin"):  # the kernels' in-launch BN-backward finalize, as its own step
            e.run_fin()
    dx.copy_(g.bfloat16())
    return dx


def conv_stem_fwd(x4, w16s, out, *, R=7, S=7, stride=2, pad=3, stats=None, patch=None):
    OC = w16s.shape[0]
    w = w16s.float().view(OC, 8, 8, 4)[:, :R, :S, :].permute(0, 3, 1, 2)
    y = _nhwc(F.conv2d(_nchw(x4.float()), w, stride=stride, padding=pad)).bfloat16()
    out.copy_(y)
    if stats is not None:
        _add_stats(stats, out)
    return out


def conv_wgrad(dy, x, dw, ws, *, R, S, stride, pad, in_scale=None, in_shift=None, relu_in=True, scale=1.0,
               accumulate=False, stem=False, tile=None, lds_pad=0, dma=-1, cnt=None, out_krsc=None, rounds=None,
               defer=None, cu_reserve=0):
    N, OH, OW, OC = dy.shape
    IC = x.shape[-1]
    xf = _act_in(x, in_scale, in_shift, relu_in)
    g = torch.nn.grad.conv2d_weight(_nchw(xf), (OC, IC, R, S), _nchw(dy.float()), stride=stride, padding=pad)
    g = g.permute(0, 2, 3, 1) * scale  # KRSC
    if stem and out_krsc is not None:  # the real input channels only (x is padded to 4)
        icr = out_krsc.numel() // (OC * R * S)
        out_krsc.copy_((g[..., :icr].reshape(-1) + (out_krsc if accumulate else 0)))
        return out_krsc
    if stem:
        full = torch.zeros(OC, 8, 8, 4, dtype=torch.float32, device=dy.device)
        full[:, :R, :S, :IC] = g
        g = full
    g = g.reshape(dw.shape)
    if accumulate:
        g = g + dw
    dw.copy_(g)
    return dw


def conv_dwfused(g, y3, coeff, wt16, y2, scale2, shift2, mean2, invstd2, bstats2, da, dw, ws, cus=0):
    """Fused bottleneck-conv3 backward = BN3-backward apply -> MASK_Y dgrad + weight gradient."""
    from types import SimpleNamespace
    dy = torch.empty_like(g)
    bn_bwd_apply(g, y3, coeff, dy, mask_mode=MASK_NONE)
    act = torch.relu(y2.float() * scale2 + shift2).bfloat16()
    epi = SimpleNamespace(mode=MASK_Y, ybn=y2, mean1=mean2, inv1=invstd2, stats1=bstats2, mbits=None, scale=scale2,
                          shift=shift2, ybn2=None, mean2=None, inv2=None, stats2=None, act_out=None)
    conv_dgrad(dy, wt16, da, R=1, S=1, stride=1, pad=0, epilogue=epi)
    conv_wgrad(dy, act, dw, ws, R=1, S=1, stride=1, pad=0)
    return da


def bn_finalize(stats, count, gamma, beta, eps, momentum, running_mean, running_var, scale, shift, save_mean,
                save_invstd):
    C = scale.numel()
    st = stats.view(-1, 2, C).double().sum(0)
    mean = st[0] / count
    var = (st[1] / count - mean * mean).clamp_min(0)
    invstd = 1.0 / torch.sqrt(var + eps)
    g = gamma.double() if gamma is not None else torch.ones_like(mean)
    b = beta.double() if beta is not None else torch.zeros_like(mean)
    scale.copy_((g * invstd).float())
    shift.copy_((b - mean * g * invstd).float())
    if save_mean is not None:
        save_mean.copy_(mean.float())
    if save_invstd is not None:
        save_invstd.copy_(invstd.float())
    if running_mean is not None and momentum > 0:
        unb = var * count / (count - 1) if count > 1 else var
        running_mean.mul_(1 - momentum).add_(momentum * mean.float())
        running_var.mul_(1 - momentum).add_(momentum * unb.float())


def bn_eval_coeff(gamma, beta, eps, running_mean, running_var, scale, shift):
    inv = torch.rsqrt(running_var + eps)
    g = gamma if gamma is not None else torch.ones_like(inv)
    b = beta if beta is not None else torch.zeros_like(inv)
    scale.copy_(g * inv)
    shift.copy_(b - running_mean * g * inv)


def channel_stats(y, stats):
    _add_stats(stats, y)


def bn_apply(y, scale, shift, out, *, res=None, res_scale=None, res_shift=None, relu=True, mbits=None, fin=None,
             res_fin=None):
    for fn in (fin, res_fin):  # (the kernel finalizes in-launch; here: the finalize first)
        if fn is not None:
            fn.run()
    f = y.float() * scale + shift
    if res is not None:
        r = res.float()
        if res_scale is not None:
            r = r * res_scale + res_shift
        f = f + r
    if relu:
        f = torch.relu(f)
    out.copy_(f.bfloat16())
    if mbits is not None:
        b = (out.reshape(-1, 8).float() > 0).to(torch.int32)
        mbits.copy_((b * (2 ** torch.arange(8, dtype=torch.int32))).sum(1).to(torch.uint8))
    return out


MASK_NONE, MASK_OUT, MASK_Y = 0, 1, 2


def _g(dout, y, mask_mode, mref, scale, shift):
    g = dout.float()
    if mask_mode == MASK_OUT:
        g = g * (mref.float() > 0)
    elif mask_mode == MASK_Y:
        g = g * ((y.float() * scale + shift) > 0)
    return g


def bn_bwd_reduce(dout, y, mean, invstd, stats, *, mask_mode, mref=None, scale=None, shift=None):
    C = y.shape[-1]
    g = _g(dout, y, mask_mode, mref, scale, shift).reshape(-1, C)
    xhat = ((y.float() - mean) * invstd).reshape(-1, C)
    st = stats.view(-1, 2, C)
    st[0, 0] += g.sum(0)
    st[0, 1] += (g * xhat).sum(0)


def bn_bwd_coeff(stats, count, gamma, mean, invstd, coeff, dgamma=None, dbeta=None, accumulate=False):
    C = mean.numel()
    st = stats.view(-1, 2, C).sum(0).float()
    s, q = st[0], st[1]
    g = gamma if gamma is not None else torch.ones_like(mean)
    sg, sgx = s / count, q / count
    k1 = g * invstd
    k2 = -g * invstd * invstd * sgx
    k3 = -g * invstd * sg + g * invstd * invstd * sgx * mean
    coeff.view(3, C).copy_(torch.stack([k1, k2, k3]))
    if dgamma is not None:
        dgamma.copy_(q + (dgamma if accumulate else 0))
    if dbeta is not None:
        dbeta.copy_(s + (dbeta if accumulate else 0))


def bn_bwd_apply(dout, y, coeff, dy, *, mask_mode, mref=None, scale=None, shift=None, gout=None, fin=None):
    if fin is not None:  # (the kernel finalizes the coefficients in-launch; here: the finalize first)
        fin.run()
    C = y.shape[-1]
    g = _g(dout, y, mask_mode, mref, scale, shift)
    if gout is not None:
        gout.copy_(g.bfloat16())
    k = coeff.view(3, C)
    dy.copy_((k[0] * g + k[1] * y.float() + k[2]).bfloat16())


def bn_bwd_apply2(g, y1, coeff1, dy1, y2, coeff2, dy2, fin1=None, fin2=None):
    bn_bwd_apply(g, y1, coeff1, dy1, mask_mode=0, fin=fin1)
    bn_bwd_apply(g, y2, coeff2, dy2, mask_mode=0, fin=fin2)


def maxpool_fwd(x, out, arg, *, K=3, stride=2, pad=1, scale=None, shift=None, relu=True, ymax=None, fin=None):
    if fin is not None:
        fin.run()
    f = x.float()
    if scale is not None:
        f = f * scale + shift
    if relu:
        f = torch.relu(f)
    N, H, W, C = f.shape
    _, P, Q, _ = out.shape
    fp = F.pad(_nchw(f), (pad, pad, pad, pad), value=-math.inf)
    xp = F.pad(_nchw(x.float()), (pad, pad, pad, pad))
    best = torch.full((N, C, P, Q), -math.inf, dtype=torch.float32, device=x.device)
    braw = torch.zeros((N, C, P, Q), dtype=torch.float32, device=x.device)
    bidx = torch.zeros((N, C, P, Q), dtype=torch.uint8, device=x.device)
    for r in range(K):
        for s in range(K):
            sl = (slice(None), slice(None), slice(r, r + stride * (P - 1) + 1, stride),
                  slice(s, s + stride * (Q - 1) + 1, stride))
            win = fp[sl]
            upd = win > best
            best = torch.where(upd, win, best)
            braw = torch.where(upd, xp[sl], braw)
            bidx = torch.where(upd, torch.full_like(bidx, r * K + s), bidx)
    out.copy_(_nhwc(best).bfloat16())
    arg.copy_(_nhwc(bidx))
    if ymax is not None:
        ymax.copy_(_nhwc(braw).bfloat16())


def maxpool_bwd(dout, arg, dx, *, K=3, stride=2, pad=1):
    N, H, W, C = dx.shape
    _, P, Q, _ = dout.shape
    acc = torch.zeros(N, C, H + 2 * pad, W + 2 * pad, dtype=torch.float32, device=dx.device)
    g = _nchw(dout.float())
    a = _nchw(arg)
    for r in range(K):
        for s in range(K):
            contrib = torch.where(a == r * K + s, g, torch.zeros_like(g))
            acc[:, :, r:r + stride * (P - 1) + 1:stride, s:s + stride * (Q - 1) + 1:stride] += contrib
    dx.copy_(_nhwc(acc[:, :, pad:pad + H, pad:pad + W]).bfloat16())


def _pool_g(dpool, arg, y, scale, shift, K, stride, pad):
    N, H, W, C = y.shape
    _, P, Q, _ = dpool.shape
    acc = torch.zeros(N, C, H + 2 * pad, W + 2 * pad, dtype=torch.float32, device=y.device)
    g = _nchw(dpool.float())
    a = _nchw(arg)
    for r in range(K):
        for s in range(K):
            acc[:, :, r:r + stride * (P - 1) + 1:stride, s:s + stride * (Q - 1) + 1:stride] += torch.where(
                a == r * K + s, g, torch.zeros_like(g))
    da = _nhwc(acc[:, :, pad:pad + H, pad:pad + W])
    return torch.where(y.float() * scale + shift > 0, da, torch.zeros_like(da))


def pool_bn_bwd_reduce(dpool, arg, y, scale, shift, mean, invstd, stats, *, K=3, stride=2, pad=1):
    C = y.shape[-1]
    g = _pool_g(dpool, arg, y, scale, shift, K, stride, pad).reshape(-1, C)
    xhat = ((y.float() - mean) * invstd).reshape(-1, C)
    st = stats.view(-1, 2, C)
    st[0, 0] += g.sum(0).double()
    st[0, 1] += (g * xhat).sum(0).double()


def pool_bn_bwd_apply(dpool, arg, y, scale, shift, coeff, dy, *, K=3, stride=2, pad=1):
    C = y.shape[-1]
    g = _pool_g(dpool, arg, y, scale, shift, K, stride, pad)
    k = coeff.view(3, C)
    dy.copy_((k[0] * g + k[1] * y.float() + k[2]).bfloat16())


def stem_bwd_fused(dpool, arg, y, scale, shift, coeff, x4, dw, ws, *, K=3, stride=2, pad=1, R=7, S=7,
                   conv_stride=2, conv_pad=3):
    """Fused stem backward = pool_bn_bwd_apply + the stem weight gradient."""
    dy = torch.empty_like(y)
    pool_bn_bwd_apply(dpool, arg, y, scale, shift, coeff, dy, K=K, stride=stride, pad=pad)
    conv_wgrad(dy, x4, dw, ws, R=R, S=S, stride=conv_stride, pad=conv_pad, stem=True)
    return dw


def avgpool_fwd(x, out):
    out.copy_(x.float().mean((1, 2)).bfloat16())


def avgpool_bwd(dout, dx):
    N, H, W, C = dx.shape
    dx.copy_((dout.float() / (H * W))[:, None, None, :].expand(N, H, W, C).bfloat16())


def softmax_ce(logits, labels, dlogits=None, loss_out=None, stats=None, smoothing=0.0, grad_scale=1.0,
               labels2=None, lam=None):
    B, C = logits.shape
    lf = logits.float()
    lse = torch.logsumexp(lf, 1)
    xl = lf.gather(1, labels[:, None]).squeeze(1)
    lm = float(lam.reshape(-1)[0]) if labels2 is not None else 1.0
    xl2 = lf.gather(1, labels2[:, None]).squeeze(1) if labels2 is not None else xl
    loss = (1 - smoothing) * (lm * (lse - xl) + (1 - lm) * (lse - xl2)) + smoothing * (lse - lf.mean(1))
    if loss_out is not None:
        loss_out.copy_(loss)
    if stats is not None:
        stats[0] += loss.sum()
        stats[1] += (lf.argmax(1) == labels).sum().float()
    if dlogits is not None:
        p = torch.softmax(lf, 1)
        t = torch.full_like(p, smoothing / C)
        t.scatter_add_(1, labels[:, None], torch.full((B, 1), (1 - smoothing) * lm, device=p.device))
        if labels2 is not None:
            t.scatter_add_(1, labels2[:, None], torch.full((B, 1), (1 - smoothing) * (1 - lm), device=p.device))
        dlogits.copy_(((p - t) * grad_scale / B).to(dlogits.dtype))


def sgd_step(p, g, v, p16=None, *, lr, momentum, dampening=0.0, weight_decay=0.0, nesterov=False, first=False,
             grad_scale_ptr=None, grad_scale=1.0, hyper=None):
    if hyper is not None:
        lr = float(hyper[0])
    gs = grad_scale * (float(grad_scale_ptr[0]) if grad_scale_ptr is not None else 1.0)
    d = g * gs + weight_decay * p
    if momentum != 0:
        if first:
            v.copy_(d)
        else:
            v.mul_(momentum).add_(d, alpha=1 - dampening)
        d = d + momentum * v if nesterov else v
    p.sub_(lr * d)
    if p16 is not None:
        p16.copy_(p.bfloat16())


def adam_step(p, g, m, v, p16=None, *, lr, beta1, beta2, eps, weight_decay, decoupled, step, grad_scale_ptr=None,
              grad_scale=1.0, hyper=None):
    bc1, bc2 = 1 - beta1 ** step, 1 - beta2 ** step
    if hyper is not None:
        lr, bc1, bc2 = float(hyper[0]), float(hyper[1]), float(hyper[2])
    gs = grad_scale * (float(grad_scale_ptr[0]) if grad_scale_ptr is not None else 1.0)
    gg = g * gs
    if decoupled:
        p.mul_(1 - lr * weight_decay)
    else:
        gg = gg + weight_decay * p
    m.mul_(beta1).add_(gg, alpha=1 - beta1)
    v.mul_(beta2).addcmul_(gg, gg, value=1 - beta2)
    p.sub_(lr * (m / bc1) / (torch.sqrt(v / bc2) + eps))
    if p16 is not None:
        p16.copy_(p.bfloat16())


def global_norm_clip_factor(g, max_norm, work):
    work.zero_()
    ss = (g.double() ** 2).sum()
    work[0:2].view(torch.float64)[0] = ss
    nrm = torch.sqrt(ss).float()
    work[2] = torch.clamp(max_norm / (nrm + 1e-6), max=1.0)
    work[3] = nrm
    return work[2:3]


def sumsq_accum(g, work):
    w = work[0:2].view(torch.float64)
    w += (g.double() ** 2).sum()


def clip_factor(work, max_norm):
    nrm = torch.sqrt(work[0:2].view(torch.float64)[0]).float()
    work[2] = torch.clamp(max_norm / (nrm + 1e-6), max=1.0)
    work[3] = nrm
    return work[2:3]


def normalize_u8(img, out, mean, std, flip=None):
    N, H, W, Cin = img.shape
    f = img.float() / 255.0
    if Cin == 1:
        f = f.expand(N, H, W, 3)
    if flip is not None:
        fl = flip.bool()[:, None, None, None]
        f = torch.where(fl, f.flip(2), f)
    m = torch.tensor(mean, device=img.device)
    s = torch.tensor(std, device=img.device)
    o = torch.zeros(N, H, W, 4, device=img.device)
    o[..., :3] = (f - m) / s
    out.copy_(o.bfloat16())


def augment_u8(img, out, boxes, mean, std, flip=None, perm=None, mixbox=None):
    if perm is not None:  # CutMix: the augmented batch, then the box pasted from sample perm[n]
        augment_u8(img, out, boxes, mean, std, flip)
        y0, y1, x0, x1 = (int(v) for v in mixbox.tolist())
        if y0 < y1 and x0 < x1:
            src = out.clone()
            out[:, y0:y1, x0:x1] = src[perm.long()][:, y0:y1, x0:x1]
        return
    N, Hin, Win, Cin = img.shape
    _, Ho, Wo, _ = out.shape
    dev = img.device
    res = torch.zeros(N, Ho, Wo, 4, device=dev)
    oy = torch.arange(Ho, device=dev).float()
    ox = torch.arange(Wo, device=dev).float()
    m = torch.tensor(mean, device=dev)
    s = torch.tensor(std, device=dev)
    for n in range(N):
        by, bx, bh, bw = (float(v) for v in boxes[n])
        oxx = (Wo - 1 - ox) if (flip is not None and int(flip[n])) else ox
        sy = (by + (oy + 0.5) * bh / Ho - 0.5).clamp(0, Hin - 1)
        sx = (bx + (oxx + 0.5) * bw / Wo - 0.5).clamp(0, Win - 1)
        y0, x0 = sy.floor().long(), sx.floor().long()
        y1, x1 = (y0 + 1).clamp(max=Hin - 1), (x0 + 1).clamp(max=Win - 1)
        wy, wx = (sy - y0)[:, None, None], (sx - x0)[None, :, None]
        im = img[n].float()
        if Cin == 1:
            im = im.expand(Hin, Win, 3)
        im = im[..., :3]
        v = ((im[y0][:, x0] * (1 - wx) + im[y0][:, x1] * wx) * (1 - wy) + (im[y1][:, x0] * (1 - wx) + im[y1][:, x1] * wx) * wy)
        res[n, ..., :3] = (v / 255.0 - m) / s
    out.copy_(res.bfloat16())


def weight_prep(master, wbuf, desc_dev, nlayers):
    d = desc_dev.view(-1, 10)
    for i in range(nlayers):
        row = d[i]
        src, fwd, tr = (int(x) for x in row[:6].view(torch.int64))
        k, rs, c = int(row[6]), int(row[7]), int(row[8])
        if tr == -2:  # stem (K, R, S, C) -> (K, 8, 8, 4) zero padded
            R, S = rs >> 4, rs & 15
            o = torch.zeros(k, 8, 8, 4, dtype=torch.bfloat16, device=wbuf.device)
            o[:, :R, :S, :c] = master[src:src + k * R * S * c].float().view(k, R, S, c).bfloat16()
            wbuf[fwd:fwd + k * 256].copy_(o.reshape(-1))
            continue
        if tr < -2:  # absolute-pointer utility entries (GPU only)
            continue
        n = k * rs * c
        w = master[src:src + n].float()
        if fwd >= 0:
            wbuf[fwd:fwd + n].copy_(w.bfloat16())
        if tr >= 0:
            wbuf[tr:tr + n].copy_(w.view(k, rs, c).permute(2, 1, 0).reshape(-1).bfloat16())


def cast_f32_bf16(x, y):
    y.copy_(x.bfloat16())


def lars_scale(p, g, seg_off, seg_len, adapt, norms, *, grad_scale, eta, weight_decay, max_len):
    for s, (o, n, a) in enumerate(zip(seg_off.tolist(), seg_len.tolist(), adapt.tolist())):
        w, d = p[o:o + n], g[o:o + n]
        d.mul_(grad_scale)
        wn, gn = w.norm(), d.norm()
        norms[2 * s], norms[2 * s + 1] = wn * wn, gn * gn
        if a:
            trust = float(eta * wn / (gn + weight_decay * wn)) if (wn > 0 and gn > 0) else 1.0
            d.add_(w, alpha=weight_decay).mul_(trust)


# ---- classifier head (csrc/head_ops.hip) ------------------------------------------------------------
def philox_u32(idx, seed: int, offset: int):
    """Philox-4x32-10 word ``idx % 4`` of counter (idx / 4 lo, idx / 4 hi, offset, 0), key seed --
    bit-identical to head_ops.hip (numpy uint64 arithmetic)."""
    import numpy as np
    idx = np.asarray(idx, dtype=np.uint64)
    M32 = np.uint64(0xFFFFFFFF)
    c0 = (idx >> np.uint64(2)) & M32
    c1 = (idx >> np.uint64(34)) & M32
    c2 = np.full_like(idx, np.uint64(offset & 0xFFFFFFFF))
    c3 = np.zeros_like(idx)
    k0, k1 = seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF
    for _ in range(10):
        p0 = np.uint64(0xD2511F53) * c0
        p1 = np.uint64(0xCD9E8D57) * c2
        n0 = (p1 >> np.uint64(32)) ^ c1 ^ np.uint64(k0)
        n1 = p1 & M32
        n2 = (p0 >> np.uint64(32)) ^ c3 ^ np.uint64(k1)
        n3 = p0 & M32
        c0, c1, c2, c3 = n0, n1, n2, n3
        k0 = (k0 + 0x9E3779B9) & 0xFFFFFFFF
        k1 = (k1 + 0xBB67AE85) & 0xFFFFFFFF
    w = idx & np.uint64(3)
    return np.where(w == 0, c0, np.where(w == 1, c1, np.where(w == 2, c2, c3)))


def dropout_mask(numel: int, p: float, seed: int, offset: int, device=None) -> torch.Tensor:
    import numpy as np
    keep = 1.0 - p
    thr = min(0xFFFFFFFF, int(round(keep * 4294967296.0)))
    u = philox_u32(np.arange(numel, dtype=np.uint64), seed, offset)
    return torch.from_numpy((u < np.uint64(thr)).astype(np.float32) / keep).to(device)


def small_gemm(A, B, out, *, ta=False, tb=False, M, N, K, alpha=1.0, bias=None, accumulate=False, dropout=None,
               ws=None):
    a = A.float().reshape(K, M).t() if ta else A.float().reshape(M, K)
    b = B.float().reshape(K, N) if tb else B.float().reshape(N, K).t()
    if dropout is not None:
        which, pd, seed, off = dropout
        src = A if which == "A" else B
        off = int(off.reshape(-1)[0]) if isinstance(off, torch.Tensor) else int(off)
        mk = dropout_mask(src.numel(), pd, int(seed), off, src.device).reshape(src.shape)
        if which == "A":
            a = (A.float() * mk).bfloat16().float().reshape(K, M).t() if ta else \
                (A.float() * mk).bfloat16().float().reshape(M, K)
        else:
            b = (B.float() * mk).bfloat16().float().reshape(K, N) if tb else \
                (B.float() * mk).bfloat16().float().reshape(N, K).t()
    r = alpha * (a @ b)
    if bias is not None:
        r = r + bias.float().reshape(1, N)
    o = out.reshape(M, N)
    if accumulate:
        r = r + o.float()
    o.copy_(r.to(out.dtype))
    return out


def colsum(x, out, accumulate=False):
    s = x.float().sum(0)
    out.copy_(out + s if accumulate else s)
    return out


def dropout(x, y, p, seed, offset):
    offset = int(offset.reshape(-1)[0]) if isinstance(offset, torch.Tensor) else int(offset)
    y.copy_((x.float() * dropout_mask(x.numel(), p, int(seed), int(offset), x.device).reshape(x.shape)).to(y.dtype))
    return y
