"""Multi-rank GPU tests: the world > 1 path (per-segment HIP graphs + comm-stream bucket
collectives + ZeRO-1) and bench.py's own rank spawning.

* RCCL at world 2 / 4 / 8: one GPU per rank; skipped unless that many devices are visible (the
  round-end 8-GPU node runs them; a one-GPU box skips them).
* gloo at world 2 on ONE GPU (both ranks on cuda:0): the same segmented-graph code path with the
  collectives on gloo, which always runs on a GPU box.

Every rank group runs in child processes started by the launcher CLI (the pytest process may have
initialised the GPU, so it only starts children; it never forks ranks itself)."""
import json
import os
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]


def _ndev() -> int:
    return torch.cuda.device_count()


def _run(cmd, env_extra=None, timeout=600):
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.update(env_extra or {})
    return subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)


def _launch(nproc, script, env_extra=None):
    cmd = [sys.executable, "-m", "dbx_distributed_pytorch_examples_amd.launch", "--nproc-per-node", str(nproc),
           os.path.join(ROOT, script)]
    return _run(cmd, env_extra)


def test_dist_check_gloo_two_ranks_one_gpu():
    r = _launch(2, "tools/dist_gpu_check.py", {"DBX_DIST_BACKEND": "gloo", "CUDA_VISIBLE_DEVICES": "0"})
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "dist_gpu_check OK: world=2 backend=gloo" in r.stdout


@pytest.mark.parametrize("comm", ["torch", "native"])
@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_dist_check_rccl(world, comm):
    """DP gradient == sum of per-rank gradients, graph == eager, ZeRO-1 == DP over RCCL, through
    c10d (comm=torch) or the framework communicator + one-graph step (comm=native). World 1 is
    the one-GPU rehearsal (one-rank RCCL group, segmented multi-rank path forced): every RCCL-only
    branch -- c10d reduce_scatter_tensor / all_gather_into_tensor in parallel/zero.py included --
    runs there."""
    if _ndev() < world:
        pytest.skip(f"RCCL world {world} needs {world} GPUs ({_ndev()} visible)")
    env = {"DBX_ENGINE": f"comm={comm}"}
    if world == 1:
        env.update({"DBX_FORCE_PG": "1", "DBX_ENGINE": f"comm={comm},segmented_graphs=1"})
    r = _launch(world, "tools/dist_gpu_check.py", env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert f"dist_gpu_check OK: world={world} backend=nccl comm={comm}" in r.stdout


def _bench_line(stdout: str) -> dict:
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, stdout[-2000:]
    return json.loads(lines[0])


def test_bench_self_launch_gloo_one_gpu():
    r = _run([sys.executable, "bench.py", "--gpus", "2", "--preset", "resnet18_cifar10", "--batch", "32",
              "--steps", "2", "--warmup", "2"], {"DBX_DIST_BACKEND": "gloo", "CUDA_VISIBLE_DEVICES": "0"})
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    d = _bench_line(r.stdout)
    assert d["n_gpus"] == 2 and d["config"]["world_size_seen"] == 2 and d["config"]["backend"] == "gloo"
    assert d["config"]["global_batch"] == 64 and d["value"] > 0


@pytest.mark.parametrize("world", [2, 8])
def test_bench_self_launch_rccl(world):
    if _ndev() < world:
        pytest.skip(f"needs {world} GPUs")
    r = _run([sys.executable, "bench.py", "--gpus", str(world), "--preset", "resnet18_cifar10", "--steps", "3",
              "--warmup", "3"])
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    d = _bench_line(r.stdout)
    assert d["n_gpus"] == world and d["config"]["world_size_seen"] == world and d["config"]["backend"] == "nccl"


def test_bench_more_gpus_than_visible_fails_loudly():
    n = _ndev() + 1
    r = _run([sys.executable, "bench.py", "--gpus", str(n), "--steps", "1", "--warmup", "0"], timeout=300)
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    assert "GPU(s) visible" in r.stderr and not r.stdout.strip()
