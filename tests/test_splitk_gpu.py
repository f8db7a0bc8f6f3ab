"""Split-K of the few-tile implicit-GEMM convs (EngineConfig splitk_wgs / splitk_min_kb; the in-launch
combine of csrc/conv_igemm_kernel.h splitk_combine): against the unsplit launch and the fp32 PyTorch
reference, bit-identical from run to run and across graph replays."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

dev = "cuda"

# N, H, W, IC, OC, R, stride, pad: the TinyImageNet layer3 / layer4 shapes at small batch
CASES = [(32, 4, 4, 1024, 256, 1, 1, 0), (32, 4, 4, 256, 256, 3, 1, 1), (16, 2, 2, 2048, 512, 1, 1, 0),
         (8, 2, 2, 512, 512, 3, 1, 1), (16, 4, 4, 512, 256, 3, 2, 1)]


def K():
    from dbx_distributed_pytorch_examples_amd.ops import kernels
    return kernels


def relerr(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


def nchw(x):
    return x.permute(0, 3, 1, 2).contiguous()


def _fwd(k, x, w, case, sc, sh):
    N, H, W, IC, OC, R, st, pad = case
    OH, OW = k.conv_out_hw(H, W, R, R, st, pad)
    out = torch.empty(N, OH, OW, OC, device=dev, dtype=torch.bfloat16)
    stats = k.new_stats(OC, dev)
    k.conv_fwd(x, w.view(OC, -1), out, R=R, S=R, stride=st, pad=pad, stats=stats, in_scale=sc, in_shift=sh,
               relu_in=True)
    return out, stats.view(-1, 2, OC).sum(0)


def _dgrad(k, dy, wt, case):
    N, H, W, IC, OC, R, st, pad = case
    dx = torch.empty(N, H, W, IC, device=dev, dtype=torch.bfloat16)
    k.conv_dgrad(dy, wt.view(IC, -1), dx, R=R, S=R, stride=st, pad=pad)
    return dx


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("prologue", [False, True])
def test_splitk_matches_unsplit_and_reference(case, prologue, engine):
    k = K()
    N, H, W, IC, OC, R, st, pad = case
    if prologue and IC > 512:
        pytest.skip("the plain BN prologue stages <= 512 channels (wider inputs arrive through the tail prologue)")
    torch.manual_seed(0)
    x = torch.randn(N, H, W, IC, device=dev).bfloat16()
    w = (torch.randn(OC, R, R, IC, device=dev) / math.sqrt(IC * R * R)).bfloat16()
    sc = sh = None
    xe = x.float()
    if prologue:
        sc = torch.rand(IC, device=dev) + 0.5
        sh = torch.randn(IC, device=dev) * 0.1
        xe = torch.relu(x.float() * sc + sh).bfloat16().float()
    OH, OW = k.conv_out_hw(H, W, R, R, st, pad)
    dy = torch.randn(N, OH, OW, OC, device=dev).bfloat16()
    wt = w.permute(3, 1, 2, 0).contiguous()
    ref = nhwc(F.conv2d(nchw(xe), w.float().permute(0, 3, 1, 2), stride=st, padding=pad))
    ref_dx = nhwc(torch.nn.grad.conv2d_input((N, IC, H, W), w.float().permute(0, 3, 1, 2), nchw(dy.float()),
                                             stride=st, padding=pad))
    engine(splitk_wgs=0)
    o0, s0 = _fwd(k, x, w, case, sc, sh)
    d0 = _dgrad(k, dy, wt, case)
    engine(splitk_wgs=4096, splitk_min_kb=1)  # as many slices as the K blocks allow
    bm, bn = k.pick_tile(N * OH * OW, OC, "fwd" if prologue else "fwd0", IC, R, st)[:2]
    assert k.conv_splitk(N * OH * OW, OC, bm, bn, 0, R * R * IC // 64)[0] > 1  # this case really splits
    o1, s1 = _fwd(k, x, w, case, sc, sh)
    d1 = _dgrad(k, dy, wt, case)
    torch.cuda.synchronize()
    assert relerr(o1, ref) < 1e-2 and relerr(d1, ref_dx) < 1e-2
    assert relerr(o1, o0) < 5e-3 and relerr(d1, d0) < 5e-3  # fp32 sums in another order, one bf16 rounding
    assert relerr(s1, s0) < 1e-3
    for _ in range(3):  # the same bits whichever slice of a tile arrives last
        o2, s2 = _fwd(k, x, w, case, sc, sh)
        d2 = _dgrad(k, dy, wt, case)
        assert torch.equal(o2, o1) and torch.equal(s2, s1) and torch.equal(d2, d1)


def test_splitk_graph_replay(engine):
    """Captured split-K launches replay with the counters the combine reset: identical to eager."""
    k = K()
    case = (32, 4, 4, 1024, 256, 1, 1, 0)
    N, H, W, IC, OC, R, st, pad = case
    torch.manual_seed(3)
    x = torch.randn(N, H, W, IC, device=dev).bfloat16()
    w = (torch.randn(OC, R, R, IC, device=dev) / math.sqrt(IC * R * R)).bfloat16()
    engine(splitk_wgs=4096, splitk_min_kb=2)
    out = torch.empty(N, H, W, OC, device=dev, dtype=torch.bfloat16)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        k.conv_fwd(x, w.view(OC, -1), out, R=1, S=1, stride=1, pad=0)  # eager: allocates the slab buffers
        eager = out.clone()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            k.conv_fwd(x, w.view(OC, -1), out, R=1, S=1, stride=1, pad=0)
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(4):
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, eager)
