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
