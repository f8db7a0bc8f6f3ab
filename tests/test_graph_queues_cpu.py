"""The HIP graph-queue setting (package __init__): DEBUG_HIP_FORCE_GRAPH_QUEUES=2 only works when it
is in the environment before the HIP runtime initialises. Importing the package after the GPU is up
must say so, and the pre-capture check must flag a value other than 1 / 2."""
import importlib
import warnings

import pytest
import torch


def _reload(monkeypatch, initialised: bool, value=None):
    import dbx_distributed_pytorch_examples_amd as pkg
    monkeypatch.setattr(torch.cuda, "is_initialized", lambda: initialised)
    if value is None:
        monkeypatch.delenv("DEBUG_HIP_FORCE_GRAPH_QUEUES", raising=False)
    else:
        monkeypatch.setenv("DEBUG_HIP_FORCE_GRAPH_QUEUES", value)
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        pkg = importlib.reload(pkg)
    return pkg, [str(x.message) for x in w]


def test_import_after_gpu_init_warns(monkeypatch):
    pkg, msgs = _reload(monkeypatch, True)
    assert any("imported after the GPU was initialised" in m for m in msgs)
    assert pkg.GRAPH_QUEUES_EFFECTIVE is None
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        assert pkg.check_graph_queues() is False
    assert any("unknown" in str(x.message) for x in w)
    monkeypatch.setenv("DBX_STRICT_GRAPH_QUEUES", "1")
    pkg._warned_queues = False
    with pytest.raises(RuntimeError):
        pkg.check_graph_queues()


def test_import_before_gpu_init_is_effective(monkeypatch):
    pkg, msgs = _reload(monkeypatch, False)
    assert not any("imported after" in m for m in msgs)
    assert pkg.GRAPH_QUEUES_EFFECTIVE == "2" and pkg.check_graph_queues()


def test_explicit_unsafe_value_is_flagged(monkeypatch):
    pkg, _ = _reload(monkeypatch, False, "4")
    assert pkg.GRAPH_QUEUES_EFFECTIVE == "4"
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        assert pkg.check_graph_queues() is False
    assert any("1 or 2 are safe" in str(x.message) for x in w)


def test_user_value_before_init_counts(monkeypatch):
    pkg, msgs = _reload(monkeypatch, True, "1")
    assert pkg.GRAPH_QUEUES_EFFECTIVE == "1" and not msgs and pkg.check_graph_queues()


@pytest.fixture(autouse=True)
def _restore():
    yield
    import dbx_distributed_pytorch_examples_amd as pkg
    import os
    os.environ["DEBUG_HIP_FORCE_GRAPH_QUEUES"] = "2"
    importlib.reload(pkg)
