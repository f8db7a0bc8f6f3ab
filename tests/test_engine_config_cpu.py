"""EngineConfig: the typed engine switches and their one environment override (DBX_ENGINE)."""
import pytest
import torch

from dbx_distributed_pytorch_examples_amd.engine_config import EngineConfig, StepPolicy, engine_env


def test_defaults_and_parse():
    c = EngineConfig()
    assert c.overlap_wgrad is None and c.comm == "native" and c.multirank_layout == "block" and c.fast
    p = EngineConfig.parse("overlap_wgrad=2, side_cu_reserve=64,lazy_join=1,comm=torch,fold_max_ratio=1.5")
    assert (p.overlap_wgrad, p.side_cu_reserve, p.lazy_join, p.comm, p.fold_max_ratio) == (2, 64, True, "torch", 1.5)
    assert EngineConfig.parse("side_defer=auto").side_defer is None  # Optional fields: back to the policy
    assert EngineConfig.parse("policy.small_step_flops=1e12").policy.small_step_flops == 1e12


@pytest.mark.parametrize("bad", ["nonsense=1", "fast=2", "overlap_wgrad", "policy.bogus=1"])
def test_parse_rejects(bad):
    with pytest.raises(ValueError):
        EngineConfig.parse(bad)


def test_current_follows_the_environment(monkeypatch):
    monkeypatch.setenv("DBX_ENGINE", "tap_prune=0")
    assert EngineConfig.current().tap_prune is False
    monkeypatch.setenv("DBX_ENGINE", "tap_prune=1,comm=torch")
    assert EngineConfig.current().tap_prune is True and EngineConfig.current().comm == "torch"
    assert engine_env(comm="native").endswith("comm=native")  # appended: the last value wins
    assert EngineConfig.parse(engine_env(comm="native")).comm == "native"
    monkeypatch.delenv("DBX_ENGINE")
    assert EngineConfig.current() == EngineConfig()


def test_step_policy_classes():
    pol = StepPolicy()
    assert pol.tiny(2e10) and pol.small(2e10) and not pol.mid(2e10)        # ResNet-18 CIFAR b256
    assert pol.mid(3.5e11) and pol.small(3.5e11) and not pol.tiny(3.5e11)  # ResNet-50 TinyImageNet b512
    assert not pol.small(8.4e12)                                           # the b1024 headline


def test_explicit_config_overrides_environment(monkeypatch):
    """A program built with an explicit EngineConfig ignores DBX_ENGINE; its None fields are resolved by
    the policy of the step size (here the patched FLOP count of the TinyImageNet class)."""
    from dbx_distributed_pytorch_examples_amd.engine.program import ResNetProgram
    from dbx_distributed_pytorch_examples_amd.models import build_model
    monkeypatch.setenv("DBX_ENGINE", "overlap_wgrad=0")
    monkeypatch.setattr(ResNetProgram, "fwd_conv_flops", lambda self: 3.5e11)
    m = build_model("resnet18", num_classes=10)
    p = ResNetProgram(m, 2, (32, 32), torch.device("cpu"), engine=EngineConfig(side_cu_reserve=96))
    assert p.overlap_wgrad and p.side_block and p.side_cu_reserve == 96 and p.dwf_cus == 128 and p.tail_main == 3
    q = ResNetProgram(m, 2, (32, 32), torch.device("cpu"))
    assert not q.overlap_wgrad  # the environment's override


@pytest.mark.parametrize("arch,size,optim,nseg", [("resnet18", 32, "sgd", -1), ("resnet50", 64, "sgd", -1),
                                                  ("resnet50", 64, "adamw", 3), ("cifar_resnet18", 32, "sgd", 2)])
def test_optimizer_in_backward_is_bit_identical(arch, size, optim, nseg, monkeypatch):
    """overlap_optimizer: each backward segment's parameters are updated right after the segment (on the
    side stream on a GPU; in program order here) -- no parameter may be read after its update within the
    step, so three steps must give the end-of-step optimizer's parameters bit for bit."""
    from dbx_distributed_pytorch_examples_amd.engine.native_trainer import NativeTrainer, OptimConfig
    from dbx_distributed_pytorch_examples_amd.models import build_model
    o = OptimConfig(lr=0.05, momentum=0.9, weight_decay=5e-4) if optim == "sgd" else \
        OptimConfig(name="adamw", lr=1e-3, weight_decay=0.01)
    out = {}
    for ov in (True, False):
        monkeypatch.setenv("DBX_ENGINE", f"overlap_optimizer={nseg if ov else 0}")
        torch.manual_seed(0)
        m = build_model(arch, num_classes=10)
        tr = NativeTrainer(m, 4, (size, size), torch.device("cpu"), optim=o, use_graphs=False)
        assert (tr.opt_ranges is not None) == ov
        if ov:  # every parameter element is covered by a segment range or a gap range
            rs = sorted(r for ph in tr.opt_ranges["per_phase"] for r in ph) + tr.opt_ranges["gaps"]
            assert sum(hi - lo for lo, hi in rs) >= tr.prog.n_params
        g = torch.Generator().manual_seed(3)
        for _ in range(3):
            tr.step(torch.randint(0, 256, (4, size, size, 3), dtype=torch.uint8, generator=g),
                    torch.randint(0, 10, (4,), generator=g))
        out[ov] = (tr.prog.master.clone(), tr.mom.clone())
    assert torch.equal(out[True][0], out[False][0]) and torch.equal(out[True][1], out[False][1])
