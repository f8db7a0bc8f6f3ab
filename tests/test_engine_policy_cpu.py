"""Engine policies: the weight-gradient side-stream modes, the per-step hyper-parameter refresh (no
copy when unchanged), and the step FLOP count."""
import pytest
import torch

from dbx_distributed_pytorch_examples_amd.engine.hyper import DeviceHyper
from dbx_distributed_pytorch_examples_amd.engine.program import ResNetProgram
from dbx_distributed_pytorch_examples_amd.models import build_model


def _flops(arch, size, batch, classes=10):
    p = ResNetProgram.__new__(ResNetProgram)  # layer table only, no buffers
    p.model, p.N, p.H, p.W = build_model(arch, num_classes=classes), batch, size, size
    p._build_layers()
    return p.fwd_conv_flops()


def test_fwd_conv_flops():
    f = _flops("resnet50", 224, 1024)
    assert abs(f / 1024 / 2 - 4.09e9) / 4.09e9 < 0.05  # ~4.1 GMAC / image of forward convolution
    assert _flops("resnet18", 32, 256) < _flops("resnet50", 64, 512) < f


def test_side_stream_defaults(monkeypatch, engine):
    """Default: one side fork per residual block; 2 = the batched side stream (one fork per backward
    segment); 1 = per-gradient forks; 0 = off."""
    for env, overlap, batch, block in ((None, True, False, True), ("2", True, True, False), ("1", True, False, False),
                                       ("0", False, False, False)):
        if env is None:
            engine(overlap_wgrad=None)
        else:
            engine(overlap_wgrad=env)
        p = ResNetProgram(build_model("resnet18", num_classes=10), 2, (32, 32), torch.device("cpu"))
        assert (p.overlap_wgrad, p.side_batch, p.side_block) == (overlap, batch, block), env


def test_device_hyper_copies_only_changes():
    t = torch.zeros(4)
    h = DeviceHyper(t)
    h.set([0.1, 1.0, 1.0, 0.0])
    assert t.tolist() == pytest.approx([0.1, 1.0, 1.0, 0.0])
    t.fill_(7.0)  # an unchanged set() does not touch the device tensor
    h.set([0.1, 1.0, 1.0, 0.0])
    assert t.tolist() == [7.0] * 4
    h.set([0.2, 0.5, 0.25, 0.0])
    assert t.tolist() == pytest.approx([0.2, 0.5, 0.25, 0.0])
    h.invalidate()
    t.fill_(0.0)
    h.set([0.2, 0.5, 0.25, 0.0])
    assert t.tolist() == pytest.approx([0.2, 0.5, 0.25, 0.0])


def test_post_launch_hook_owner_scoped_cancel():
    """ops.kernels.set_post_launch: a program cancels only its own pending deferred side launch."""
    from dbx_distributed_pytorch_examples_amd.ops import kernels as K

    class P:
        def launch(self):
            pass
    a, b = P(), P()
    try:
        K.set_post_launch(a.launch)
        K.set_post_launch(None, owner=b.launch)   # another program's cancel: kept
        assert K._POST_LAUNCH == a.launch
        K.set_post_launch(None, owner=a.launch)   # its own: cancelled
        assert K._POST_LAUNCH is None
        K.set_post_launch(b.launch)
        K.set_post_launch(None)                   # unconditional cancel
        assert K._POST_LAUNCH is None
    finally:
        K.set_post_launch(None)


def test_side_stream_defaults_by_step_size(monkeypatch, engine):
    """The default side stream forks per residual block with the deferred launch and lazy joins, the
    last block's tail and the stem weight gradient on the main stream, the downsample forwards on the
    side stream; the CU reservation from 50 GFLOP of forward conv work up; an explicit
    overlap_wgrad wins. (The step size is patched: the real ones need GPU-sized buffers.)"""
    m = build_model("resnet18", num_classes=10)
    monkeypatch.setattr(ResNetProgram, "fwd_conv_flops", lambda self: 1e11)
    p = ResNetProgram(m, 2, (32, 32), torch.device("cpu"))
    assert (p.side_block, p.side_batch, p.side_defer, p.lazy_join, p.side_cu_reserve) == (True, False, True, True, 128)
    assert p.ds_fwd_side
    assert (p.block_tail_main, p.stem_wg_main) == (2, True)
    monkeypatch.setattr(ResNetProgram, "fwd_conv_flops", lambda self: 1e10)
    p = ResNetProgram(m, 2, (32, 32), torch.device("cpu"))
    assert p.ds_fwd_side and p.block_tail_main == 2
    assert (p.side_block, p.side_batch, p.side_defer, p.lazy_join, p.side_cu_reserve) == (True, False, True, True, 0)
    monkeypatch.setattr(ResNetProgram, "fwd_conv_flops", lambda self: 1e12)
    p = ResNetProgram(m, 2, (32, 32), torch.device("cpu"))
    assert p.ds_fwd_side and (p.block_tail_main, p.stem_wg_main) == (2, True)
    engine(overlap_wgrad="2")
    p = ResNetProgram(m, 2, (32, 32), torch.device("cpu"))
    assert (p.side_block, p.side_batch, p.side_defer, p.lazy_join, p.stem_wg_main) == (False, True, False, False, False)


@pytest.mark.parametrize("flops,fin_in,coeff_in,nshard", [
    (2.0e10, True, True, 4),     # CIFAR class: consumer-side forward finalize kept
    (3.5e11, False, True, 4),    # TinyImageNet class: standalone finalize launches (profiles/r6_tiny_fin/)
    (8.4e12, False, False, None),  # headline class: NSHARD shards, standalone finalizes
])
def test_small_step_finalize_policy(monkeypatch, engine, flops, fin_in, coeff_in, nshard):
    """Round-6 policy: the consumer-side forward BN finalize only for the launch-bound CIFAR class;
    4 statistics shards and the in-apply backward finalize for both small classes."""
    from dbx_distributed_pytorch_examples_amd.engine import program as P
    from dbx_distributed_pytorch_examples_amd.ops import kernels as K
    engine(fin_in=None, coeff_in=None, nshard=None)
    monkeypatch.setattr(P.ResNetProgram, "fwd_conv_flops", lambda self: flops)
    p = ResNetProgram(build_model("resnet18", num_classes=10), 2, (32, 32), torch.device("cpu"))
    assert (p.fin_in, p.coeff_in) == (fin_in, coeff_in)
    assert p.nshard == (nshard if nshard is not None else K.NSHARD)


def test_splitk_and_sweep_defaults():
    """Defaults measured in round 6: split-K slices of >= 8 K blocks (profiles/r6_tiny_knobs/), the
    sweep forward from one 128-row block per CU, the dgrad sweep off (profiles/r6_sweep/)."""
    from dbx_distributed_pytorch_examples_amd.engine_config import EngineConfig
    c = EngineConfig()
    assert (c.splitk_wgs, c.splitk_min_kb) == (512, 8)
    assert c.sweep_fwd and not c.sweep_dgrad and c.sweep_min_tiles_per_cu == 1.0
