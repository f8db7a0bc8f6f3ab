"""Build the native extension in-tree: ``python -m dbx_distributed_pytorch_examples_amd.build_ext``.

Compiles every ``csrc/*.hip`` for gfx950 with hipcc and the pybind11 bindings, links
``_C<EXT_SUFFIX>`` next to this file (the .so travels to the GPU box with the snapshot; the
git history stays source-only). Incremental: objects newer than their sources are reused.
Environment: ``DBX_ARCH`` (default gfx950), ``DBX_HIPCC`` (default /opt/rocm/bin/hipcc),
``DBX_DEBUG=1`` builds the separate variant ``_C_variant_debug`` with ``-g -DDBX_DEBUG``: the
``DBX_DCHECK`` device checks (common.h) on the conv kernels' gather / scatter offsets then print the
failing condition, block and thread instead of letting an out-of-range offset read zeros or write
past a tensor; load it with ``DBX_EXT_VARIANT=debug`` (the production ``_C`` is never replaced).
"""
from __future__ import annotations

import glob
import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "build")


def _hipcc() -> str:
    return os.environ.get("DBX_HIPCC", "/opt/rocm/bin/hipcc")


def _pybind_includes():
    import pybind11
    return [pybind11.get_include(), sysconfig.get_paths()["include"]]


def ext_path(variant: str = "") -> str:
    """``_C<suffix>``; an A/B variant build is ``_C_variant_<name><suffix>`` (loaded by setting
    ``DBX_EXT_VARIANT=<name>``, see ops/_ext.py) so two kernel versions can be timed in one box."""
    stem = "_C" + (f"_variant_{variant}" if variant else "")
    return os.path.join(HERE, stem + sysconfig.get_config_var("EXT_SUFFIX"))


def _newer(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(verbose: bool = False, jobs: int = 8, variant: str = "", defines=()) -> str:
    arch = os.environ.get("DBX_ARCH", "gfx950")
    if os.environ.get("DBX_DEBUG") == "1" and not variant:
        variant = "debug"
    bdir = BUILD if not variant else BUILD + "_" + variant
    os.makedirs(bdir, exist_ok=True)
    headers = glob.glob(os.path.join(CSRC, "*.h"))
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip"))) + [os.path.join(CSRC, "bindings.cpp")]
    extra_srcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    dbg = ["-g", "-DDBX_DEBUG"] if os.environ.get("DBX_DEBUG") == "1" else []
    common = ["-O3", "-fPIC", "-std=c++17", f"-I{CSRC}"] + [f"-I{p}" for p in _pybind_includes()] + dbg + \
        [f"-D{d}" for d in defines]
    objs, cmds = [], []
    for s in srcs + extra_srcs:
        o = os.path.join(bdir, os.path.basename(s) + ".o")
        objs.append(o)
        if _newer(o, [s] + headers):
            if s.endswith(".hip"):
                cmd = [_hipcc(), f"--offload-arch={arch}", "-munsafe-fp-atomics", "-Wno-inline-asm", "-c", s, "-o", o] + common
            else:
                cmd = [_hipcc(), "-c", s, "-o", o] + common + ["-fvisibility=hidden"]
            cmds.append(cmd)

    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        return r.stderr

    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for err in ex.map(run, cmds):
            if verbose and err.strip():
                print(err)
    out = ext_path(variant)
    if _newer(out, objs):
        link = [_hipcc(), "-shared", "-fPIC", f"--offload-arch={arch}", "-o", out] + objs + [
            "-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib"]
        run(link)
    return out


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("-v", action="store_true")
    ap.add_argument("--variant", default="", help="A/B build name (-> _C_variant_<name>)")
    ap.add_argument("-D", dest="defines", action="append", default=[], help="preprocessor define for the variant")
    a = ap.parse_args()
    print(build(verbose=a.v, variant=a.variant, defines=a.defines))
