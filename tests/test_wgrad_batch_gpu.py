"""Deferred split-K weight-gradient reductions (ops/kernels.py ReduceBatch, csrc/conv_igemm.hip
dbx_wgrad_reduce_multi): a batch of weight gradients reduced by two launches at its end is
bit-identical to each gradient's own reduce (one- and two-level), in eager execution."""
import pytest
import torch

from dbx_distributed_pytorch_examples_amd.ops import kernels as K

pytestmark = pytest.mark.gpu

# (N, H, IC, OC, R, rounds): split depths from none to > 8 splits (the two-level reduction)
CASES = [(8, 14, 64, 64, 3, 2.0), (16, 8, 128, 256, 1, 4.0), (64, 4, 256, 256, 3, 8.0), (32, 7, 64, 128, 1, 1.0),
         (128, 2, 512, 512, 3, 16.0), (256, 1, 512, 512, 1, 32.0)]


def test_batched_reduce_matches_per_gradient_reduce():
    torch.manual_seed(0)
    ws = torch.empty(64 << 20, device="cuda")
    arena = torch.empty(256 << 20, device="cuda")
    ops = []
    for (N, H, IC, OC, R, rounds) in CASES:
        x = torch.randn(N, H, H, IC, device="cuda").bfloat16()
        dy = torch.randn(N, H, H, OC, device="cuda").bfloat16()
        ops.append((dy, x, R, rounds, OC * R * R * IC))
    outs = []
    for deferred in (False, True):
        batch = K.ReduceBatch(arena) if deferred else None
        dws = []
        for i, (dy, x, R, rounds, n) in enumerate(ops):
            dw = torch.full((n,), 0.5, device="cuda")  # accumulate onto a non-zero gradient for odd i
            K.conv_wgrad(dy, x, dw, ws, R=R, S=R, stride=1, pad=R // 2, scale=0.25, accumulate=bool(i % 2),
                         rounds=rounds, defer=batch)
            dws.append(dw)
        if batch is not None:
            assert batch.jobs, "nothing was deferred"
            batch.flush()
        torch.cuda.synchronize()
        outs.append(dws)
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    # and against fp32 torch for one case
    dy, x, R, _, _ = ops[1]
    ref = torch.einsum("nhwk,nhwc->kc", dy.float(), x.float()).reshape(-1) * 0.25 + 0.5
    assert (outs[1][1] - ref).abs().max() / ref.abs().max() < 1e-2


@pytest.mark.parametrize("arch,size,batch", [("cifar_resnet18", 32, 64), ("resnet50", 64, 32)])
def test_program_deferred_reduce_bit_identical(arch, size, batch, monkeypatch, engine):
    """Whole training steps (eager warm-ups, capture, replays) with the batched reduce == without,
    bit for bit, twice (a run-to-run difference would show in one of the two)."""
    import copy
    from dbx_distributed_pytorch_examples_amd.engine.native_trainer import NativeTrainer, OptimConfig
    from dbx_distributed_pytorch_examples_amd.models import build_model
    torch.manual_seed(0)
    m0 = build_model(arch, num_classes=10)
    ms = [copy.deepcopy(m0) for _ in range(3)]
    ts = []
    for m, flag in zip(ms, ("0", "1", "1")):
        engine(defer_reduce=flag)
        ts.append(NativeTrainer(m, batch, (size, size), torch.device("cuda"), optim=OptimConfig(lr=0.05)))
    assert ts[1].prog.defer_reduce and not ts[0].prog.defer_reduce
    g = torch.Generator().manual_seed(1)
    for i in range(6):
        img = torch.randint(0, 256, (batch, size, size, 3), dtype=torch.uint8, generator=g).cuda()
        lab = torch.randint(0, 10, (batch,), generator=g).cuda()
        for t in ts:
            t.step(img, lab)
        m = [t.read_metrics()[0] for t in ts]
        assert m[0] == m[1] == m[2], (i, m)
    assert ts[1].prog.wred_arena.numel() > 0  # the warm-up steps sized the arena before the capture
    for t in ts[1:]:
        assert torch.equal(ts[0].prog.master, t.prog.master)
