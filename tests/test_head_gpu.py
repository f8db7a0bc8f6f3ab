"""Native classifier head (csrc/head_ops.hip: fc GEMMs with bias / Philox dropout, bias-gradient
column sums) and the CutMix pieces (box paste in augment_u8, mixed soft targets in softmax_ce),
each against a plain PyTorch fp32 reference of the same op."""
import pytest
import torch

from dbx_distributed_pytorch_examples_amd.ops import kernels as K
from dbx_distributed_pytorch_examples_amd.ops import reference as R

pytestmark = pytest.mark.gpu


def _bf(*shape, scale=1.0):
    return (torch.randn(*shape, device="cuda") * scale).bfloat16()


@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, True), (True, False)])
@pytest.mark.parametrize("M,N,Kd", [(1024, 1000, 2048), (256, 10, 512), (37, 70, 33)])
def test_small_gemm_layouts_vs_fp32(ta, tb, M, N, Kd):
    torch.manual_seed(M + N + Kd)
    A = _bf(Kd, M) if ta else _bf(M, Kd)
    B = _bf(Kd, N) if tb else _bf(N, Kd)
    bias = torch.randn(N, device="cuda")
    out = torch.empty(M, N, device="cuda")
    K.small_gemm(A, B, out, ta=ta, tb=tb, M=M, N=N, K=Kd, bias=bias, alpha=0.5)
    a = A.float().t() if ta else A.float()
    b = B.float() if tb else B.float().t()
    ref = 0.5 * (a @ b) + bias
    torch.cuda.synchronize()
    err = (out - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-5, err  # bf16 x bf16 products are exact in fp32; only summation order differs


def test_small_gemm_bf16_out_accumulate_and_bias16():
    torch.manual_seed(1)
    M, N, Kd = 300, 200, 256
    A, B = _bf(M, Kd), _bf(N, Kd)
    out = _bf(M, N)
    base = out.float().clone()
    b16 = _bf(N)
    K.small_gemm(A, B, out, M=M, N=N, K=Kd, bias=b16, accumulate=True)
    ref = base + A.float() @ B.float().t() + b16.float()
    assert torch.allclose(out.float(), ref, atol=0.1, rtol=1e-2)


@pytest.mark.parametrize("which", ["A", "B"])
def test_small_gemm_dropout_mask_matches_reference_philox(which):
    torch.manual_seed(2)
    M, N, Kd = 128, 96, 512
    A, B = _bf(M, Kd), _bf(Kd, N)
    out = torch.empty(M, N, device="cuda")
    spec = (which, 0.5, 1234567, 42)
    K.small_gemm(A, B, out, tb=True, M=M, N=N, K=Kd, dropout=spec)
    ref = torch.empty(M, N)
    R.small_gemm(A.cpu(), B.cpu(), ref, tb=True, M=M, N=N, K=Kd, dropout=spec)
    assert torch.allclose(out.cpu(), ref, atol=1e-3, rtol=1e-4)
    # the dropout kernel regenerates the same mask (the forward's h for the weight gradient)
    src = A if which == "A" else B
    y = torch.empty_like(src)
    K.dropout(src, y, 0.5, 1234567, 42)
    yr = torch.empty(src.shape, dtype=torch.bfloat16)
    R.dropout(src.cpu(), yr, 0.5, 1234567, 42)
    assert torch.equal(y.cpu(), yr)
    kept = (y != 0).float().mean().item()
    assert 0.45 < kept < 0.55


@pytest.mark.parametrize("M,N", [(1000, 1000), (256, 10), (37, 70)])
def test_colsum(M, N):
    x = _bf(M, N)
    out = torch.empty(N, device="cuda")
    K.colsum(x, out)
    assert torch.allclose(out, x.float().sum(0), atol=1e-3, rtol=1e-4)
    base = out.clone()
    K.colsum(x, out, accumulate=True)
    assert torch.allclose(out, 2 * base, atol=1e-3, rtol=1e-4)


def test_softmax_ce_cutmix_soft_targets_vs_reference():
    torch.manual_seed(3)
    B, C = 64, 1000
    logits = torch.randn(B, C, device="cuda").bfloat16()
    y = torch.randint(0, C, (B,), device="cuda")
    y2 = torch.randint(0, C, (B,), device="cuda")
    lam = torch.tensor([0.37], device="cuda")
    dl = torch.empty_like(logits)
    st = torch.zeros(2, device="cuda", dtype=torch.float64)
    K.softmax_ce(logits, y, dl, None, st, smoothing=0.1, labels2=y2, lam=lam)
    lf = logits.float()
    t = 0.9 * (0.37 * torch.nn.functional.one_hot(y, C) + 0.63 * torch.nn.functional.one_hot(y2, C)) + 0.1 / C
    ref_loss = -(t * torch.log_softmax(lf, 1)).sum(1)
    ref_dl = (torch.softmax(lf, 1) - t) / B
    torch.cuda.synchronize()
    assert abs(st[0].item() - ref_loss.sum().item()) < 1e-3 * ref_loss.sum().item()
    assert torch.allclose(dl.float(), ref_dl, atol=2e-5, rtol=2e-2)


def test_augment_cutmix_paste_vs_reference():
    torch.manual_seed(4)
    N, H, W = 8, 40, 40
    img = torch.randint(0, 256, (N, H, W, 3), dtype=torch.uint8, device="cuda")
    out = torch.empty(N, 32, 32, 4, device="cuda", dtype=torch.bfloat16)
    boxes = torch.tensor([[2.0, 3.0, 32.0, 32.0]] * N, device="cuda")
    flip = (torch.arange(N, device="cuda") % 2).to(torch.uint8)
    perm = torch.randperm(N, device="cuda").int()
    box = torch.tensor([5, 21, 9, 30], device="cuda", dtype=torch.int32)
    mean, std = (0.4, 0.45, 0.5), (0.25, 0.2, 0.22)
    K.augment_u8(img, out, boxes, mean, std, flip, perm=perm, mixbox=box)
    ref = torch.empty(N, 32, 32, 4, dtype=torch.bfloat16)
    R.augment_u8(img.cpu(), ref, boxes.cpu(), mean, std, flip.cpu(), perm=perm.cpu(), mixbox=box.cpu())
    assert (out.cpu().float() - ref.float()).abs().max() < 0.05
    plain = torch.empty_like(out)
    K.augment_u8(img, plain, boxes, mean, std, flip)
    assert torch.equal(out[:, 5:21, 9:30], plain[perm.long()][:, 5:21, 9:30])  # pasted pixels
    assert torch.equal(out[:, :5], plain[:, :5])                              # untouched rows


def test_native_trainer_cutmix_trains():
    """CutMix stays on the native engine: the loss of a fixed batch falls over 30 steps."""
    from dbx_distributed_pytorch_examples_amd.engine.native_trainer import NativeTrainer, OptimConfig
    from dbx_distributed_pytorch_examples_amd.models import build_model
    torch.manual_seed(0)
    tr = NativeTrainer(build_model("resnet18", num_classes=10), 64, (32, 32), torch.device("cuda"),
                       optim=OptimConfig(name="adam", lr=1e-3, weight_decay=0.0), label_smoothing=0.1,
                       cutmix_alpha=1.0)
    img = torch.randint(0, 256, (64, 32, 32, 3), dtype=torch.uint8, device="cuda")
    lab = torch.randint(0, 10, (64,), device="cuda")
    losses = []
    for i in range(30):
        tr.step(img, lab)
        if i % 10 == 9:
            losses.append(tr.read_metrics()[0] / (10 * 64))
    assert all(l == l for l in losses) and losses[-1] < losses[0], losses


@pytest.mark.parametrize("ta,tb", [(False, True), (True, False), (False, False)])
@pytest.mark.parametrize("M,N,Kd", [(512, 200, 2048), (32, 1000, 2048), (200, 2048, 512), (37, 70, 1111)])
def test_small_gemm_split_k_matches_single_pass(ta, tb, M, N, Kd):
    """Split-K (few output tiles, long K: the TinyImageNet / small-batch fc shapes) sums the
    partials in split order after one pass: same result as the fp32 reference; fp32 + bias + alpha,
    bf16 out + accumulate, and the dropout operand all go through the reduce epilogue."""
    torch.manual_seed(M * 7 + N + Kd)
    A = _bf(Kd, M) if ta else _bf(M, Kd)
    B = _bf(Kd, N) if tb else _bf(N, Kd)
    bias = torch.randn(N, device="cuda")
    ws = torch.empty(8 * max(M * N, 1), device="cuda")
    sk = K.head_splitk(M, N, Kd, ws.numel())
    out = torch.empty(M, N, device="cuda")
    K.small_gemm(A, B, out, ta=ta, tb=tb, M=M, N=N, K=Kd, bias=bias, alpha=0.5, ws=ws)
    a = A.float().t() if ta else A.float()
    b = B.float() if tb else B.float().t()
    ref = 0.5 * (a @ b) + bias
    torch.cuda.synchronize()
    err = (out - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-5, (sk, err)
    o16 = _bf(M, N)
    base = o16.float().clone()
    K.small_gemm(A, B, o16, ta=ta, tb=tb, M=M, N=N, K=Kd, accumulate=True, ws=ws)
    assert torch.allclose(o16.float(), base + a @ b, atol=0.25, rtol=1e-2), sk
    if not ta and tb:
        spec = ("A", 0.5, 99, 7)
        K.small_gemm(A, B, out, tb=True, M=M, N=N, K=Kd, dropout=spec, ws=ws)
        one = torch.empty_like(out)
        K.small_gemm(A, B, one, tb=True, M=M, N=N, K=Kd, dropout=spec)
        assert torch.allclose(out, one, atol=1e-4, rtol=1e-4), sk
