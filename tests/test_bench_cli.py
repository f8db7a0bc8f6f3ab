"""bench.py contract on CPU: self-launched ranks (gloo), world/--gpus mismatch is an error, the
JSON line carries the world size the process group formed and per-preset metric labels."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.timeout(600)


def _run(args, env_extra=None, timeout=500):
    env = dict(os.environ)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd="/tmp", env=env,
                          capture_output=True, text=True, timeout=timeout)


def _line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_self_launch_two_ranks_gloo_cpu():
    r = _run(["--gpus", "2", "--preset", "resnet18_cifar10", "--batch", "4", "--steps", "1", "--warmup", "0"],
             {"DBX_DIST_BACKEND": "gloo"})
    assert r.returncode == 0, r.stderr[-3000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == 2 and d["config"]["world_size_seen"] == 2 and d["config"]["backend"] == "gloo"
    assert d["config"]["global_batch"] == 8 and d["config"]["per_gpu_batch"] == 4  # explicit --batch wins
    assert "ResNet-18 CIFAR-10" in d["metric"] and "CIFAR-10" in d["config"]["model"]
    assert d["vs_baseline"] is None  # not the preset's batch: no comparable baseline


def test_world_mismatch_is_an_error():
    # under a launcher environment that says world 1, --gpus 2 must not report a number
    r = _run(["--gpus", "2", "--steps", "1"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 3 and "refusing" in r.stderr and not r.stdout.strip()


def test_no_gpus_visible_fails_before_spawning():
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("two GPUs visible: --gpus 2 would run")
    r = _run(["--gpus", "2", "--steps", "1"], {"DBX_DIST_BACKEND": ""})
    assert r.returncode == 3 and "GPU(s) visible" in r.stderr


def test_two_rank_bench_checks_replicas():
    """World > 1: bench.py checks after warm-up and after the timed steps that every rank holds
    bit-identical parameters (the check runs in the gloo rehearsal of the driver's N-GPU command)."""
    r = _run(["--gpus", "2", "--preset", "resnet18_cifar10", "--batch", "4", "--steps", "1", "--warmup", "1"],
             {"DBX_DIST_BACKEND": "gloo"})
    assert r.returncode == 0, r.stderr[-3000:]
    assert "replicas in sync after warm-up" in r.stderr and "replicas in sync after the timed steps" in r.stderr
    _line(r.stdout)


def test_diverged_replica_refuses_to_report():
    r = _run(["--gpus", "2", "--preset", "resnet18_cifar10", "--batch", "4", "--steps", "1", "--warmup", "1"],
             {"DBX_DIST_BACKEND": "gloo", "DBX_FAULT": "1:0:diverge"})
    assert r.returncode == 4 and "diverged" in r.stderr, r.stderr[-2000:]
    assert not any(ln.startswith("{") for ln in r.stdout.splitlines())


def test_stalled_rank_ends_the_bench_within_the_timeout():
    """A rank that stops in warm-up (DBX_FAULT hang) must not leave the N-GPU bench blocked until the
    driver's timeout: the watchdog names the phase and the job exits 75 within --phase-timeout
    (with the fresh-rank re-run switched off, --comm-fallback 0)."""
    import time
    t0 = time.time()
    r = _run(["--gpus", "2", "--preset", "resnet18_cifar10", "--batch", "4", "--steps", "1", "--warmup", "2",
              "--phase-timeout", "10", "--comm-fallback", "0"], {"DBX_DIST_BACKEND": "gloo", "DBX_FAULT": "1:1:hang"})
    assert r.returncode == 75, r.stderr[-2000:]
    assert "[comm-watchdog]" in r.stderr and "phase 'warmup'" in r.stderr
    assert not any(ln.startswith("{") for ln in r.stdout.splitlines())
    assert time.time() - t0 < 120


def test_hung_self_launched_ranks_are_remeasured_on_fresh_ranks():
    """bench.py --gpus N (self-launched): a collective hang in warm-up ends the ranks with exit 75; the
    GPU-free parent starts fresh ranks once on the c10d step (comm=torch; the injected fault only
    fires on attempt 0) and the JSON line carries the reason in ``comm_fallback``."""
    r = _run(["--gpus", "2", "--preset", "resnet18_cifar10", "--batch", "4", "--steps", "1", "--warmup", "2",
              "--phase-timeout", "60"], {"DBX_DIST_BACKEND": "gloo", "DBX_FAULT": "1:1:comm_hang"})
    assert r.returncode == 0, r.stderr[-3000:]
    assert "[comm-watchdog]" in r.stderr and "re-running 2 fresh ranks" in r.stderr
    d = _line(r.stdout)
    assert "exit 75" in d["comm_fallback"] and d["n_gpus"] == 2


def test_hung_torchrun_ranks_are_remeasured_on_fresh_ranks():
    """The driver's form, ``torch.distributed.run ... bench.py --gpus N``: each torchrun rank supervises a
    child (GPU-free supervisor); a hang in warm-up ends the children (75), the supervisors agree through
    torchrun's agent store and re-run every rank once on a fresh rendezvous with comm=torch."""
    import socket
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    env = dict(os.environ, DBX_DIST_BACKEND="gloo", DBX_FAULT="1:1:comm_hang")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                        "--gpus", "2", "--preset", "resnet18_cifar10", "--batch", "4", "--steps", "1", "--warmup", "2",
                        "--phase-timeout", "60"],
                       cwd="/tmp", env=env, capture_output=True, text=True, timeout=500)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "[comm-watchdog]" in r.stderr and "[supervise]" in r.stderr
    d = _line(r.stdout)
    assert "exit 75" in d["comm_fallback"] and d["config"]["world_size_seen"] == 2


def test_rccl_summary_parses_the_ring_log(tmp_path):
    sys.path.insert(0, ROOT)
    import bench
    log = tmp_path / "r.log"
    log.write_text("host:1:1 [0] NCCL INFO RCCL version 2.26.6-develop:abc\n"
                   "host:1:1 [0] NCCL INFO Channel 00/16 :    0   1   2   3   4   5   6   7\n"
                   "host:1:1 [0] NCCL INFO Channel 01/16 :    0   7   6   5   4   3   2   1\n"
                   "host:1:1 [0] NCCL INFO 16 coll channels, 16 collnet channels, 0 nvls channels\n")
    d = bench.rccl_summary(str(log))
    assert d["version"].startswith("2.26.6") and d["channels"] == 16 and d["coll_channels"] == 16
    assert d["rings"][0] == "0 1 2 3 4 5 6 7" and len(d["rings"]) == 2


def test_diverged_one_graph_step_is_remeasured_on_c10d(monkeypatch, capsys, engine):
    """The one-graph multi-rank step failing its replica check (on every rank: the check gathers all
    checksums) is rebuilt on the c10d collectives (comm=torch) and measured again; a divergence
    on the c10d path (or without the framework communicator) still ends the run with 4."""
    sys.path.insert(0, ROOT)
    import bench
    calls = []

    def fake(args, info, wd, build_step, ddist, fault):
        from dbx_distributed_pytorch_examples_amd.engine_config import EngineConfig
        calls.append(EngineConfig.current().comm)
        if len(calls) == 1:
            return 4, 0.0, {"_native_comm": True}
        return 0, 1.0, {"grad_collectives": "c10d"}

    engine(comm=None)
    monkeypatch.setenv("DBX_ENGINE", "")  # (bench.main's fallback rewrites it: restored after the test)
    monkeypatch.setattr(bench, "_measure", fake)
    assert bench.main(["--steps", "1", "--warmup", "0", "--preset", "resnet18_cifar10"]) == 0
    assert calls == ["native", "torch"]
    d = _line(capsys.readouterr().out)
    assert d["config"]["grad_collectives"] == "c10d" and "_native_comm" not in d["config"]
    calls.clear()
    monkeypatch.setattr(bench, "_measure", lambda *a: (calls.append(1), (4, 0.0, {"_native_comm": False}))[1])
    assert bench.main(["--steps", "1", "--warmup", "0", "--preset", "resnet18_cifar10"]) == 4 and calls == [1]


def test_torchrun_teardown_takes_the_supervised_children_along():
    """When torchrun tears the group down (here: SIGTERM to the whole launcher), no supervised rank
    child may survive it: the supervisors kill their children's process groups on SIGTERM and the
    children die with their parent (PR_SET_PDEATHSIG) -- otherwise a hung rank would keep the GPU."""
    import signal
    import socket
    import time

    import psutil
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    env = dict(os.environ, DBX_DIST_BACKEND="gloo", DBX_FAULT="0:0:hang")
    env.pop("WORLD_SIZE", None)
    p = subprocess.Popen([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                          "--gpus", "2", "--preset", "resnet18_cifar10", "--batch", "4", "--steps", "1", "--warmup", "2",
                          "--phase-timeout", "600"], cwd="/tmp", env=env, stdout=subprocess.DEVNULL,
                         stderr=subprocess.DEVNULL, start_new_session=True)
    try:
        deadline, kids = time.time() + 180, []
        while time.time() < deadline:  # wait for both ranks' supervised children
            kids = [c for c in psutil.Process(p.pid).children(recursive=True)
                    if "bench.py" in " ".join(c.cmdline()) and c.environ().get("DBX_SUPERVISED_CHILD")]
            if len(kids) >= 2:
                break
            time.sleep(1)
        assert len(kids) >= 2, "supervised children did not start"
        time.sleep(5)
        os.killpg(p.pid, signal.SIGTERM)
        p.wait(60)
        gone, alive = psutil.wait_procs(kids, timeout=60)
        assert not alive, f"children outlived the launcher: {[c.pid for c in alive]}"
    finally:
        if p.poll() is None:
            os.killpg(p.pid, signal.SIGKILL)
