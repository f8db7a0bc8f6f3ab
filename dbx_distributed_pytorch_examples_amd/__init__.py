"""dbx_distributed_pytorch_examples_amd — MI355X-native distributed image-classification training.

A from-scratch re-design of alexxx-db/dbx-distributed-pytorch-examples for AMD Instinct
MI355X (gfx950): NHWC bf16 ResNet programs on hand-written HIP/CDNA4 kernels, one process per
GPU over RCCL/xGMI, one launcher in place of the reference's five launcher shims.
"""
import os as _os

__version__ = "0.1.0"

# HIP graph launch runs a captured graph's parallel branches on extra queues. With the runtime's
# default queue count, launching the framework's step graphs (main stream + side-stream weight
# gradients / comm-stream buckets) crashed the HIP runtime on the host in hipGraphLaunch for some
# graph shapes and stream assignments (torch's bundled HIP 7.0; a stream-pool walk past its end).
# Two queues -- the main chain plus one for the overlapped branches -- never crashed and keep the
# full overlap throughput (headline 16.46k, CIFAR 252.9k, TinyImageNet 95.5k img/s), one queue
# crashes never either but serializes the branches (-1.2 % / -6.8 % / -7.8 %): profiles/r4_final2/.
# Read by the HIP runtime when it initialises, so set here, before any device use; an explicit
# setting in the environment wins.
import sys as _sys

_QUEUES = "DEBUG_HIP_FORCE_GRAPH_QUEUES"
_user_queues = _os.environ.get(_QUEUES)
_torch = _sys.modules.get("torch")
try:  # torch not imported yet -> the GPU cannot have been initialised
    _gpu_before_import = bool(_torch is not None and _torch.cuda.is_initialized())
except Exception:  # noqa: BLE001
    _gpu_before_import = False
_os.environ.setdefault(_QUEUES, "2")
# what the HIP runtime actually read: our default (or the user's value) when the GPU comes up after
# this import; when it was up before, only a value the process already had can have been read
GRAPH_QUEUES_EFFECTIVE = _os.environ[_QUEUES] if not _gpu_before_import else _user_queues
if _gpu_before_import and _user_queues is None:
    import warnings as _w
    _w.warn(f"{__name__} was imported after the GPU was initialised: {_QUEUES}=2 (the setting that avoids a "
            "HIP runtime crash in hipGraphLaunch for the framework's step graphs) came too late for this "
            "process; import the package before any GPU use or export the variable "
            "(profiles/r4_final2/README.md)", RuntimeWarning, stacklevel=2)


def check_graph_queues() -> bool:
    """Before a capture whose graph has parallel branches: True when the runtime runs with the graph
    queue count known not to crash (1 or 2); otherwise warn (once) -- or raise with
    ``DBX_STRICT_GRAPH_QUEUES=1``."""
    global _warned_queues
    ok = GRAPH_QUEUES_EFFECTIVE in ("1", "2")
    if not ok and not _warned_queues:
        msg = (f"{_QUEUES} is {GRAPH_QUEUES_EFFECTIVE or 'unknown (the GPU was initialised before this package was imported)'}: "
               "step graphs with parallel branches crashed the HIP runtime in hipGraphLaunch with other values "
               "(profiles/r4_final2/README.md); 1 or 2 are safe")
        if _os.environ.get("DBX_STRICT_GRAPH_QUEUES", "0") == "1":
            raise RuntimeError(msg)
        import warnings as _w
        _w.warn(msg, RuntimeWarning, stacklevel=2)
        _warned_queues = True
    return ok


_warned_queues = False
