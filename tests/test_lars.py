"""LARS (large-batch SGD for the global-batch-8192 config):
the native ``lars_scale`` kernel (+ plain SGD) against the torch ``LARS`` optimizer and its
PyTorch reference, on CPU and on the MI355X."""
import copy

import pytest
import torch
import torch.nn.functional as F

from dbx_distributed_pytorch_examples_amd.engine.autograd_trainer import LARS
from dbx_distributed_pytorch_examples_amd.engine.native_trainer import NativeTrainer, OptimConfig
from dbx_distributed_pytorch_examples_amd.models import build_model
from dbx_distributed_pytorch_examples_amd.ops import kernels as K
from dbx_distributed_pytorch_examples_amd.ops import reference as R


def _segments(shapes, dev="cpu", seed=0):
    g = torch.Generator().manual_seed(seed)
    offs, lens, adapt, o = [], [], [], 0
    for s in shapes:
        n = int(torch.tensor(s).prod())
        offs.append(o)
        lens.append(n)
        adapt.append(int(len(s) > 1))
        o += (n + 15) // 16 * 16
    p = torch.randn(o, generator=g)
    gr = torch.randn(o, generator=g) * 0.1
    it = lambda v: torch.tensor(v, dtype=torch.int32, device=dev)
    return p.to(dev), gr.to(dev), it(offs), it(lens), it(adapt), max(lens)


SHAPES = [(64, 3, 7, 7), (64,), (64,), (256, 64, 1, 1), (256,), (1000, 2048), (1000,), (5,), (2048, 512, 3, 3)]


def test_reference_lars_matches_torch_optimizer():
    p, g, off, ln, ad, mx = _segments(SHAPES)
    params = [torch.nn.Parameter(p[o:o + n].clone().view(s)) for o, n, s in zip(off.tolist(), ln.tolist(), SHAPES)]
    opt = LARS(params, lr=0.5, momentum=0.9, weight_decay=1e-4, trust_coefficient=0.02)
    for q, o, n in zip(params, off.tolist(), ln.tolist()):
        q.grad = (g[o:o + n] * 0.5).view(q.shape).clone()
    opt.step()
    pm, gm, v = p.clone(), g.clone(), torch.zeros_like(p)
    R.lars_scale(pm, gm, off, ln, ad, torch.zeros(2 * len(SHAPES)), grad_scale=0.5, eta=0.02, weight_decay=1e-4,
                 max_len=mx)
    R.sgd_step(pm, gm, v, lr=0.5, momentum=0.9, weight_decay=0.0, first=False)
    for q, o, n in zip(params, off.tolist(), ln.tolist()):
        assert torch.allclose(q.detach().reshape(-1), pm[o:o + n], atol=1e-6, rtol=1e-5)


@pytest.mark.parametrize("clip", [0.0, 0.5])
def test_native_lars_step_matches_autograd_lars_cpu(clip):
    """One native-program LARS step (CPU reference ops) moves every parameter like torch LARS on the
    autograd gradients of the same batch (cosine of the updates). With grad_clip the global-norm
    clip applies before the trust ratios on both engines (clip_grad_norm_ + LARS)."""
    torch.manual_seed(0)
    model = build_model("resnet18", num_classes=10)
    ref = copy.deepcopy(model).train()
    o = OptimConfig(name="lars", lr=2.0, momentum=0.9, weight_decay=1e-4, trust_coefficient=0.02, grad_clip=clip)
    tr = NativeTrainer(model, 8, (32, 32), torch.device("cpu"), optim=o, use_graphs=False)
    before = {k: v.detach().clone() for k, v in model.named_parameters()}
    gen = torch.Generator().manual_seed(1)
    img = torch.randint(0, 256, (8, 32, 32, 3), dtype=torch.uint8, generator=gen)
    lab = torch.randint(0, 10, (8,), generator=gen)
    tr.step(img, lab)
    x = tr.prog.x4[..., :3].float().permute(0, 3, 1, 2).contiguous()
    opt = LARS(ref.parameters(), lr=2.0, momentum=0.9, weight_decay=1e-4, trust_coefficient=0.02)
    F.cross_entropy(ref(x), lab).backward()
    if clip:
        torch.nn.utils.clip_grad_norm_(ref.parameters(), clip)
    opt.step()
    nr = dict(ref.named_parameters())
    ratios = []  # update-norm ratios of the non-adapted (BN / bias) parameters: scaled by the clip
    for name, prm in model.named_parameters():
        d_nat = (prm.detach() - before[name]).flatten()
        d_ref = (nr[name].detach() - before[name]).flatten()
        if prm.dim() == 1:
            ratios.append((d_nat.norm() / d_ref.norm()).item())
        cos = (d_nat @ d_ref / (d_nat.norm() * d_ref.norm() + 1e-20)).item()
        assert cos > (0.85 if prm.dim() > 1 else 0.75), (name, cos)  # bf16 program vs fp32 autograd grads
        if prm.dim() > 1:  # the trust ratio fixes the update norm: eta * lr * |w| (up to wd)
            assert 0.8 < d_nat.norm() / d_ref.norm() < 1.25, name
    assert 0.9 < sorted(ratios)[len(ratios) // 2] < 1.1, ratios  # global norm ~109: clip 0.5 is active


@pytest.mark.gpu
def test_lars_kernel_matches_reference_gpu():
    p, g, off, ln, ad, mx = _segments(SHAPES, dev="cuda")
    pr, gr = p.cpu(), g.cpu()
    K.lars_scale(p, g, off, ln, ad, torch.zeros(K.LARS_MAX_BLOCKS * 2 * len(SHAPES), device="cuda", dtype=torch.float64), grad_scale=0.125, eta=0.001,
                 weight_decay=5e-5, max_len=mx)
    R.lars_scale(pr, gr, off.cpu(), ln.cpu(), ad.cpu(), torch.zeros(2 * len(SHAPES)), grad_scale=0.125, eta=0.001,
                 weight_decay=5e-5, max_len=mx)
    torch.cuda.synchronize()
    assert torch.allclose(g.cpu(), gr, atol=1e-7, rtol=1e-4), (g.cpu() - gr).abs().max()


@pytest.mark.gpu
def test_native_lars_resnet50_graph_step_gpu():
    """The captured native step with LARS on ResNet-50 (graph replay follows the LR schedule): loss
    falls on a fixed batch."""
    torch.manual_seed(0)
    dev = torch.device("cuda:0")
    tr = NativeTrainer(build_model("resnet50", num_classes=10), 32, (64, 64), dev,
                       optim=OptimConfig(name="lars", lr=1.0, momentum=0.9, weight_decay=5e-5, trust_coefficient=0.01),
                       use_graphs=True)
    gen = torch.Generator().manual_seed(2)
    img = torch.randint(0, 256, (32, 64, 64, 3), dtype=torch.uint8, generator=gen).to(dev)
    lab = torch.randint(0, 10, (32,), generator=gen).to(dev)
    losses = []
    for _ in range(12):
        tr.step(img, lab)
        losses.append(tr.read_metrics()[0] / 32)
    assert all(l == l for l in losses) and losses[-1] < losses[0], losses


@pytest.mark.gpu
def test_lars_scale_bit_reproducible():
    """fp64 atomics for the per-segment norms: two launches give identical trust ratios."""
    import torch
    from dbx_distributed_pytorch_examples_amd.ops import kernels as K
    torch.manual_seed(0)
    n = [300000, 4096, 65536]
    p0 = torch.randn(sum(n), device="cuda")
    g0 = torch.randn(sum(n), device="cuda")
    off = torch.tensor([0, n[0], n[0] + n[1]], dtype=torch.int32, device="cuda")
    ln = torch.tensor(n, dtype=torch.int32, device="cuda")
    ad = torch.tensor([1, 0, 1], dtype=torch.int32, device="cuda")
    outs = []
    for _ in range(3):
        g = g0.clone()
        norms = torch.zeros(K.LARS_MAX_BLOCKS * 6, device="cuda", dtype=torch.float64)
        K.lars_scale(p0, g, off, ln, ad, norms, grad_scale=0.25, eta=1e-3, weight_decay=1e-4, max_len=max(n))
        outs.append((g, norms))
    for g, nm in outs[1:]:
        assert torch.equal(g, outs[0][0]) and torch.equal(nm, outs[0][1])
