"""Loader for the in-tree native extension ``_C`` (HIP kernels for gfx950).

Policy: on a machine with a GPU the extension is REQUIRED — every GPU op in this package runs
on it, and a missing/broken build raises instead of silently falling back to stock PyTorch
(set ``DBX_ALLOW_TORCH_FALLBACK=1`` to opt into the slow reference ops explicitly). On CPU-only
hosts the same ops run their PyTorch reference implementations (used by the unit tests).
``torch`` is imported first so the HIP runtime torch bundles (libamdhip64.so.7) is the one
the extension binds to.
"""
from __future__ import annotations

import importlib
import importlib.util
import os
import sysconfig

import torch  # noqa: F401  (must precede the extension: shared HIP runtime)

_C = None
_ERR = None


def _try_load():
    global _C, _ERR
    if _C is not None or _ERR is not None:
        return _C
    try:
        variant = os.environ.get("DBX_EXT_VARIANT", "")
        if variant:  # A/B kernel builds (build_ext --variant NAME): same module, other binary
            path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                f"_C_variant_{variant}" + sysconfig.get_config_var("EXT_SUFFIX"))
            spec = importlib.util.spec_from_file_location("dbx_distributed_pytorch_examples_amd._C", path)
            _C = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(_C)
        else:
            _C = importlib.import_module("dbx_distributed_pytorch_examples_amd._C")
    except Exception as e:  # pragma: no cover - depends on build state
        _ERR = e
    return _C


def available() -> bool:
    return _try_load() is not None


def C():
    """Return the extension module or raise (GPU paths call this)."""
    m = _try_load()
    if m is None:
        raise RuntimeError(
            "dbx native extension (_C) is not built/loadable: "
            f"{_ERR!r}. Build it with `python -m dbx_distributed_pytorch_examples_amd.build_ext`.")
    return m


def allow_fallback() -> bool:
    return os.environ.get("DBX_ALLOW_TORCH_FALLBACK", "0") == "1"


def use_native(t: torch.Tensor) -> bool:
    """True when ``t`` lives on a GPU and the HIP kernels must be used."""
    if not t.is_cuda:
        return False
    if available():
        return True
    if allow_fallback():
        return False
    C()  # raises with the load error
    return False


def stream_ptr() -> int:
    return torch.cuda.current_stream().cuda_stream


def build_if_needed(verbose: bool = False) -> str:
    from ..build_ext import build
    return build(verbose=verbose)
