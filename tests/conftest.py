import os
import sys

import pytest

# (the HIP graph-queue setting the package applies at import, before any test touches the device:
# dbx_distributed_pytorch_examples_amd/__init__.py)
os.environ.setdefault("DEBUG_HIP_FORCE_GRAPH_QUEUES", "2")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_addoption(parser):
    parser.addoption("--memlog", action="store_true", help="print free device memory around each GPU test")


@pytest.fixture
def engine(monkeypatch):
    """Set engine switches (engine_config.EngineConfig fields) for one test through DBX_ENGINE:
    ``engine(fold_min_elems=0, fuse_dw=False)``; a later call adds to / overrides earlier ones and
    ``None`` drops a field back to its default."""
    state = {}

    def set_(**kw):
        for k, v in kw.items():
            if v is None:
                state.pop(k, None)
            else:
                state[k] = int(v) if isinstance(v, bool) else v
        if state:
            monkeypatch.setenv("DBX_ENGINE", ",".join(f"{k}={v}" for k, v in state.items()))
        else:
            monkeypatch.delenv("DBX_ENGINE", raising=False)
    monkeypatch.delenv("DBX_ENGINE", raising=False)
    return set_


def engine_spec(**kw) -> str:
    """A DBX_ENGINE value (for subprocess environments)."""
    return ",".join(f"{k}={int(v) if isinstance(v, bool) else v}" for k, v in kw.items())


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")
    config.addinivalue_line("markers", "slow: long-running")


def pytest_collection_modifyitems(config, items):
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no GPU on this host")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(autouse=True)
def _gpu_release(request):
    """After every GPU test: collect the test's trainers / programs (reference cycles keep them, their
    captured graphs and the graphs' private memory pools alive until a GC pass) and return the
    cached memory, so one test's graphs and buffers do not pile up under the next ones.
    (--memlog prints the device's free memory before and after each test.)"""
    yield
    if "gpu" not in request.keywords:
        return
    import gc

    import torch
    if not torch.cuda.is_available():
        return
    log = request.config.getoption("--memlog")
    if log:
        f0, tot = torch.cuda.mem_get_info()
    gc.collect()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    if log:
        f1, _ = torch.cuda.mem_get_info()
        print(f"\n[memlog] {request.node.nodeid}: free {f0 / 2**30:.1f} -> {f1 / 2**30:.1f} GiB of "
              f"{tot / 2**30:.1f}", flush=True)
