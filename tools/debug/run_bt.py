"""Run a Python script under the native SIGSEGV backtrace handler (tools/debug/segv_bt.c),
re-installed before every graph replay (the GPU runtime installs handlers of its own):
python tools/debug/run_bt.py <script.py> [args...]"""
import ctypes
import os
import runpy
import sys

_lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libsegv_bt.so"))
_lib.segv_bt_install()
import torch  # noqa: E402

_replay = torch.cuda.CUDAGraph.replay


def _replay_bt(self):
    _lib.segv_bt_install()
    return _replay(self)


torch.cuda.CUDAGraph.replay = _replay_bt
sys.argv = sys.argv[1:]
runpy.run_path(sys.argv[0], run_name="__main__")
