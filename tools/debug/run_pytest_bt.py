"""pytest under a native SIGSEGV backtrace handler (tools/debug/segv_bt.c), re-installed before every
test (the GPU runtime installs handlers of its own when it initialises): usage
python tools/debug/run_pytest_bt.py <pytest args>"""
import ctypes
import os
import sys

_lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libsegv_bt.so"))
_lib.segv_bt_install()
import pytest  # noqa: E402


class _Plugin:
    @pytest.hookimpl(tryfirst=True)
    def pytest_runtest_call(self, item):
        _lib.segv_bt_install()


sys.exit(pytest.main(["-p", "no:faulthandler"] + sys.argv[1:], plugins=[_Plugin()]))
