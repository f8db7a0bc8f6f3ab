"""Eight-wave conv kernel (csrc/conv_fast.hip, tile (256, bn, 4)): bit-identical outputs to the
four-wave implicit-GEMM kernel (same K order -> the same fp32 sums), BN statistics equal to the fp64
sums of the stored outputs, row-tail masking, the full-rounds batch split, and the program's
materialised-input path -- each also against a plain fp32 PyTorch reference of the op."""
import math

import pytest
import torch
import torch.nn.functional as F

from dbx_distributed_pytorch_examples_amd.ops import kernels as K

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _no_splitk(engine):
    """These compare kernels bit for bit against the four-wave implicit-GEMM launch, which splits the K
    loop of few-tile launches (splitk_wgs; its own tests: test_splitk_gpu.py): compare unsplit launches."""
    engine(splitk_wgs=0)


def _stats_total(st, C):
    return st.view(K.NSHARD, 2, C).sum(0)


@pytest.mark.parametrize("N,H,C,Kc,R,bn", [(20, 14, 256, 256, 3, 256), (9, 7, 512, 512, 3, 256),
                                           (12, 14, 256, 1024, 1, 256), (20, 14, 128, 128, 3, 128)])
def test_fast_fwd_matches_four_wave_and_fp32(N, H, C, Kc, R, bn):
    torch.manual_seed(N + C)
    pad = R // 2
    x = torch.randn(N, H, H, C, device="cuda").bfloat16()
    w = (torch.randn(Kc, R * R * C, device="cuda") / math.sqrt(C * R * R)).bfloat16()
    y0, y1 = (torch.empty(N, H, H, Kc, device="cuda", dtype=torch.bfloat16) for _ in range(2))
    s0, s1 = K.new_stats(Kc, "cuda"), K.new_stats(Kc, "cuda")
    K.conv_fwd(x, w, y0, R=R, S=R, stride=1, pad=pad, stats=s0, tile=(128, 128, 0))
    K.conv_fwd(x, w, y1, R=R, S=R, stride=1, pad=pad, stats=s1, tile=(256, bn, 4))
    assert torch.equal(y0, y1)  # M = N*H*W is not a multiple of 256: row tail masked
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().view(Kc, R, R, C).permute(0, 3, 1, 2), padding=pad)
    ref = ref.permute(0, 2, 3, 1)
    assert (y1.float() - ref).abs().max() / ref.abs().max() < 1e-2
    yf = y1.double().view(-1, Kc)
    tot = torch.stack([yf.sum(0), (yf * yf).sum(0)])
    assert torch.allclose(_stats_total(s1, Kc), tot, rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("epi,accum,bn", [(0, False, 256), (1, True, 256), (2, False, 128), (2, True, 128)])
def test_fast_dgrad_epilogues_match_four_wave(epi, accum, bn):
    torch.manual_seed(epi * 7 + accum)
    N, H, C, Kc, R = 10, 14, 256, 256, 3
    dy = torch.randn(N, H, H, Kc, device="cuda").bfloat16()
    wt = (torch.randn(C, R * R * Kc, device="cuda") / math.sqrt(Kc * R * R)).bfloat16()
    ybn = torch.randn(N, H, H, C, device="cuda").bfloat16()
    mean, inv = torch.randn(C, device="cuda") * 0.1, torch.rand(C, device="cuda") + 0.5
    sc, sh = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.1
    mb = K.pack_mask_bits(torch.randn(N, H, H, C, device="cuda"))
    add = torch.randn(N, H, H, C, device="cuda").bfloat16()
    outs = []
    for tile in ((128, 128, 2), (256, bn, 4)):
        dx = torch.empty(N, H, H, C, device="cuda", dtype=torch.bfloat16)
        st = K.new_stats(C, "cuda")
        act = torch.empty_like(dx)
        e = (None if epi == 0 else K.BNBwdEpilogue(K.MASK_OUT, ybn, mean, inv, st, mbits=mb) if epi == 1 else
             K.BNBwdEpilogue(K.MASK_Y, ybn, mean, inv, st, scale=sc, shift=sh, act_out=act))
        K.conv_dgrad(dy, wt, dx, R=R, S=R, stride=1, pad=1, tile=tile, epilogue=e, addsrc=add if accum else None)
        outs.append((dx, _stats_total(st, C), act))
    (d0, s0, a0), (d1, s1, a1) = outs
    assert torch.equal(d0, d1)
    if epi:
        assert torch.allclose(s0, s1, rtol=1e-5, atol=1e-3)  # fp32 per-tile partials differ with the tile
    if epi == 2:
        assert torch.equal(a0, a1)


def test_fast_batch_split_covers_every_image():
    """More tiles than CUs but not a multiple: full rounds on the eight-wave kernel, the leftover
    images on four-wave tiles -- the same output as one four-wave launch."""
    P = K.num_cus()
    H, C, Kc = 14, 256, 256
    N = (P * 256 // (H * H)) + 37  # > one full round of 256-row tiles, plus a remainder
    assert 0 < K.fast_split(N, H * H, Kc, 256) < N
    torch.manual_seed(5)
    x = torch.randn(N, H, H, C, device="cuda").bfloat16()
    w = (torch.randn(Kc, 9 * C, device="cuda") / 48).bfloat16()
    y0, y1 = (torch.empty(N, H, H, Kc, device="cuda", dtype=torch.bfloat16) for _ in range(2))
    s0, s1 = K.new_stats(Kc, "cuda"), K.new_stats(Kc, "cuda")
    K.conv_fwd(x, w, y0, R=3, S=3, stride=1, pad=1, stats=s0, tile=(128, 128, 0))
    K.conv_fwd(x, w, y1, R=3, S=3, stride=1, pad=1, stats=s1, tile=(256, 256, 4))
    assert torch.equal(y0, y1)
    assert torch.allclose(_stats_total(s0, Kc), _stats_total(s1, Kc), rtol=1e-5, atol=1e-3)


def test_program_materialised_fast_path_matches_prologue_path(monkeypatch):
    """The program's eight-wave path (forward materialises relu(bn1(y1)) for the 3x3 conv, backward
    skips the write-back) trains the same as the BN-prologue path (fp32 parameter trajectories agree
    to bf16 noise)."""
    from dbx_distributed_pytorch_examples_amd.engine import program as prog_mod
    from dbx_distributed_pytorch_examples_amd.engine.native_trainer import NativeTrainer, OptimConfig
    from dbx_distributed_pytorch_examples_amd.models import build_model
    calls = {"n": 0}
    orig = K.pick_tile

    def pick(M, OC, mode="fwd", K_in=0, R=0, stride=1, use_table=True):
        if mode == "fwd0" and R == 3 and use_table and OC % 128 == 0:  # force the eight-wave entry
            calls["n"] += 1
            return (256, 256 if OC % 256 == 0 else 128, 4)
        return orig(M, OC, mode, K_in, R, stride, use_table)
    res = {}
    for fast in (False, True):
        monkeypatch.setattr(K, "pick_tile", pick if fast else orig)
        torch.manual_seed(0)
        tr = NativeTrainer(build_model("resnet50", num_classes=100), 16, (64, 64), torch.device("cuda"),
                           optim=OptimConfig(lr=0.05))
        assert any(any(b.mat) for b in tr.prog.blocks) == fast
        g = torch.Generator().manual_seed(1)
        for _ in range(3):
            tr.step(torch.randint(0, 256, (16, 64, 64, 3), dtype=torch.uint8, generator=g).cuda(),
                    torch.randint(0, 100, (16,), generator=g).cuda())
        torch.cuda.synchronize()
        res[fast] = tr.prog.master.clone()
    assert calls["n"] > 0
    rel = ((res[True] - res[False]).norm() / res[False].norm()).item()
    assert rel < 1e-3, rel
