"""One RCCL-native launcher for all five of the reference's launcher styles.

The reference reaches multi-GPU through five different shims: Databricks
``TorchDistributor(num_processes, local_mode=True, use_gpu=True).run(fn, **kw)``
(`01_torch_distributor/01_basic_torch_distributor.py:360-367`), ``DeepspeedTorchDistributor(numGpus,
nnodes, localMode).run(fn, **kw)`` (`02_deepspeed/01_cifar_deepspeed_resnet.py:102-109`), Composer's
in-process Trainer, Accelerate, and Ray ``TorchTrainer`` (`05_ray/01_fashion_mnist_pytorch_ray.ipynb:247-262`).
They all reduce to "start one process per GPU with RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set,
run a function, hand rank 0's result back". :class:`Launcher` does exactly that, natively:

* one process per GPU (``spawn``; each rank pins ``hipSetDevice(LOCAL_RANK)`` via dist.init);
* rank 0's return value is shipped back (tensors/modules moved to CPU first — the reference
  pickles a live GPU module back to the driver, `02_cifar_torch_distributor_resnet.py:346`);
* failure detection: a rank that exits non-zero or raises fails the whole job promptly (its
  traceback is re-raised in the parent), and a progress watchdog kills the job when any rank's
  heartbeat (``utils.fault.heartbeat()``, called by the training loops every step) stalls for
  ``heartbeat_timeout`` seconds (e.g. a rank wedged in a collective);
* elastic-style restarts: ``max_restarts`` re-launches all ranks; training entrypoints resume
  from the latest checkpoint (``DBX_RESTART_COUNT`` tells them which attempt this is);
* fault injection for tests: ``DBX_FAULT="rank:step:kind"`` (kind = exit | raise | hang | nan).

Safety rule of this machine pool: a process that has initialised the GPU must never exec
another program, so the launcher refuses to spawn from a parent that has touched HIP.
CLI (torchrun-like): ``python -m dbx_distributed_pytorch_examples_amd.launch --nproc-per-node 8 train.py ...``
(or ``... --nproc-per-node 8 -m dbx_distributed_pytorch_examples_amd.train.cli ...``)
"""
from __future__ import annotations

import argparse
import os
import shutil
import socket
import subprocess
import sys
import tempfile
import time
import traceback
from typing import Any, Callable, Dict, List, Optional

import multiprocessing as mp


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _gpu_touched() -> bool:
    m = sys.modules.get("torch")
    if m is None:
        return False
    try:
        return bool(m.cuda.is_initialized())
    except Exception:
        return False


def to_cpu(obj: Any) -> Any:
    """Recursively move tensors / modules to CPU so they can cross the process boundary."""
    import torch
    if isinstance(obj, torch.nn.Module):
        return obj.cpu()
    if isinstance(obj, torch.Tensor):
        return obj.detach().cpu()
    if isinstance(obj, dict):
        return {k: to_cpu(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        t = [to_cpu(v) for v in obj]
        return type(obj)(t) if not hasattr(obj, "_fields") else type(obj)(*t)
    return obj


class LaunchError(RuntimeError):
    pass


def _worker(payload: bytes, rank: int, env: Dict[str, str], conn) -> None:
    import cloudpickle
    os.environ.update(env)
    try:
        fn, args, kwargs = cloudpickle.loads(payload)
        res = fn(*args, **kwargs)
        if rank == 0:
            conn.send(("ok", cloudpickle.dumps(to_cpu(res))))
        else:
            conn.send(("ok", None))
    except BaseException as e:  # noqa: BLE001 - report everything to the parent
        try:
            conn.send(("err", f"rank {rank}: {type(e).__name__}: {e}\n{traceback.format_exc()}"))
        except Exception:
            pass
        conn.close()
        os._exit(1)
    conn.close()


class Launcher:
    def __init__(self, num_processes: int = 1, nnodes: int = 1, node_rank: int = 0,
                 master_addr: str = "127.0.0.1", master_port: Optional[int] = None,
                 use_gpu: Optional[bool] = None, max_restarts: int = 0,
                 heartbeat_timeout: Optional[float] = None, env: Optional[Dict[str, str]] = None,
                 start_method: str = "spawn", timeout: Optional[float] = None):
        if num_processes < 1:
            raise ValueError("num_processes must be >= 1")
        self.nproc = num_processes
        self.nnodes, self.node_rank = nnodes, node_rank
        self.master_addr = master_addr
        self.master_port = master_port
        self.use_gpu = use_gpu
        self.max_restarts = max_restarts
        self.hb_timeout = heartbeat_timeout
        self.extra_env = dict(env or {})
        self.start_method = start_method
        self.timeout = timeout
        self.attempts = 0

    def _env(self, local_rank: int, port: int, hb_dir: str, attempt: int) -> Dict[str, str]:
        world = self.nproc * self.nnodes
        e = {
            "RANK": str(self.node_rank * self.nproc + local_rank),
            "LOCAL_RANK": str(local_rank),
            "WORLD_SIZE": str(world),
            "LOCAL_WORLD_SIZE": str(self.nproc),
            "GROUP_RANK": str(self.node_rank),
            "MASTER_ADDR": self.master_addr,
            "MASTER_PORT": str(port),
            "DBX_HEARTBEAT_DIR": hb_dir,
            "DBX_RESTART_COUNT": str(attempt),
            "HSA_ENABLE_IPC_MODE_LEGACY": os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"),
        }
        if self.use_gpu is False:
            e["DBX_FORCE_CPU"] = "1"
        e.update(self.extra_env)
        return e

    def _watch(self, procs: List, conns: List, hb_dir: str) -> Any:
        t0 = time.time()
        result, errors = None, []
        done = [False] * len(procs)
        while not all(done):
            for i, (p, c) in enumerate(zip(procs, conns)):
                if done[i]:
                    continue
                if c.poll():
                    try:
                        status, data = c.recv()
                    except EOFError:
                        status, data = "err", f"rank {i}: pipe closed"
                    if status == "ok":
                        if i == 0:
                            result = data
                    else:
                        errors.append(data)
                    done[i] = True
                elif not p.is_alive():
                    if p.exitcode != 0:
                        from .parallel.comm_guard import EXIT_COMM_FAILURE
                        why = " (collective failure: comm watchdog)" if p.exitcode == EXIT_COMM_FAILURE else ""
                        errors.append(f"rank {i}: exited with code {p.exitcode}{why}")
                    done[i] = True
            if errors:
                break
            if self.hb_timeout:
                stale = _stale_ranks(hb_dir, len(procs), self.hb_timeout)
                if stale:
                    errors.append(f"watchdog: no progress from rank(s) {stale} for {self.hb_timeout}s")
                    break
            if self.timeout and time.time() - t0 > self.timeout:
                errors.append(f"job exceeded timeout {self.timeout}s")
                break
            time.sleep(0.05)
        if errors:
            for p in procs:
                if p.is_alive():
                    p.terminate()
            for p in procs:
                p.join(5)
                if p.is_alive():
                    p.kill()
            raise LaunchError("\n".join(errors))
        for p in procs:
            p.join()
        return result

    def run(self, fn: Callable, *args, **kwargs) -> Any:
        """Run ``fn(*args, **kwargs)`` on every rank; return rank 0's result."""
        import cloudpickle
        if _gpu_touched():
            raise LaunchError("refusing to spawn ranks from a process that has already initialised the GPU; "
                              "launch before any torch.cuda call (torch.cuda.device_count() is fine)")
        payload = cloudpickle.dumps((fn, args, kwargs))
        ctx = mp.get_context(self.start_method)
        last_err = None
        for attempt in range(self.max_restarts + 1):
            self.attempts = attempt + 1
            port = self.master_port or _free_port()
            hb_dir = tempfile.mkdtemp(prefix="dbx_hb_")
            procs, conns = [], []
            try:
                for lr in range(self.nproc):
                    parent, child = ctx.Pipe(duplex=False)
                    p = ctx.Process(target=_worker, args=(payload, lr, self._env(lr, port, hb_dir, attempt), child),
                                    daemon=False)
                    p.start()
                    child.close()
                    procs.append(p)
                    conns.append(parent)
                res = self._watch(procs, conns, hb_dir)
                return cloudpickle.loads(res) if res is not None else None
            except LaunchError as e:
                last_err = e
                print(f"[launch] attempt {attempt + 1}/{self.max_restarts + 1} failed:\n{e}", file=sys.stderr)
            finally:
                shutil.rmtree(hb_dir, ignore_errors=True)
        raise last_err


def _stale_ranks(hb_dir: str, n: int, timeout: float) -> List[int]:
    now = time.time()
    stale = []
    for r in range(n):
        f = os.path.join(hb_dir, f"rank{r}")
        if os.path.exists(f) and now - os.path.getmtime(f) > timeout:
            stale.append(r)
    return stale


# ----------------------------------------------------------------------------------------
# reference-compatible facades
# ----------------------------------------------------------------------------------------
class TorchDistributor(Launcher):
    """``TorchDistributor(num_processes=N, local_mode=True, use_gpu=True).run(fn, *args, **kw)``."""

    def __init__(self, num_processes: int = 1, local_mode: bool = True, use_gpu: bool = True, **kw):
        if not local_mode:
            kw.setdefault("nnodes", int(os.environ.get("DBX_NNODES", "1")))
        super().__init__(num_processes=num_processes, use_gpu=use_gpu, **kw)


class DeepspeedTorchDistributor(Launcher):
    """``DeepspeedTorchDistributor(numGpus=N, nnodes=1, localMode=True, deepspeedConfig=cfg).run(fn, **kw)``.

    Unlike the reference (which comments the config out, `02_deepspeed/01_cifar_deepspeed_resnet.py:108`),
    a ``deepspeedConfig`` given here IS applied: it is exported to the ranks as ``DBX_DEEPSPEED_CONFIG``
    (JSON) and picked up by ``train.train()`` / ``config.from_deepspeed``.
    """

    def __init__(self, numGpus: int = 1, nnodes: int = 1, localMode: bool = True, deepspeedConfig=None,
                 useGpu: bool = True, **kw):
        env = dict(kw.pop("env", {}) or {})
        if deepspeedConfig is not None:
            import json
            env["DBX_DEEPSPEED_CONFIG"] = json.dumps(deepspeedConfig)
        super().__init__(num_processes=numGpus, nnodes=nnodes, use_gpu=useGpu, env=env, **kw)
        self.deepspeed_config = deepspeedConfig


# ----------------------------------------------------------------------------------------
# CLI: torchrun-like script launcher (subprocesses; the parent never touches the GPU)
# ----------------------------------------------------------------------------------------
def run_subprocess_ranks(nproc: int, cmd: List[str], nnodes: int = 1, node_rank: int = 0,
                         master_addr: str = "127.0.0.1", master_port: Optional[int] = None,
                         max_restarts: int = 0, heartbeat_timeout: Optional[float] = None,
                         env: Optional[Dict[str, str]] = None) -> int:
    """Start ``cmd`` (an argv list, e.g. ``[sys.executable, "bench.py", ...]``) once per local rank
    with the torchrun environment set, watch the ranks, and return 0 when every rank exits 0.

    A rank that fails ends the whole attempt (the others are terminated); ``max_restarts`` re-runs
    all ranks. Used by the CLI below and by ``bench.py --gpus N`` when it is not already under a
    launcher. The caller must not have initialised the GPU (children are fork+exec'd)."""
    if _gpu_touched():
        raise LaunchError("refusing to spawn ranks from a process that has already initialised the GPU")
    L = Launcher(nproc, nnodes, node_rank, master_addr, master_port,
                 max_restarts=max_restarts, heartbeat_timeout=heartbeat_timeout, env=env)
    code = 1
    for attempt in range(max_restarts + 1):
        port = master_port or _free_port()
        hb_dir = tempfile.mkdtemp(prefix="dbx_hb_")
        procs = []
        for lr in range(nproc):
            e = dict(os.environ)
            e.update(L._env(lr, port, hb_dir, attempt))
            procs.append(subprocess.Popen(list(cmd), env=e))
        failed = None
        while True:
            codes = [p.poll() for p in procs]
            bad = [i for i, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                failed = f"rank(s) {bad} exited with {[codes[i] for i in bad]}"
                code = max(c for c in codes if c not in (None, 0))  # the worst rank's code (defined for any order)
                break
            if all(c == 0 for c in codes):
                break
            if L.hb_timeout:
                stale = _stale_ranks(hb_dir, len(procs), L.hb_timeout)
                if stale:
                    failed = f"watchdog: rank(s) {stale} made no progress for {L.hb_timeout}s"
                    code = 124
                    break
            time.sleep(0.1)
        if failed:
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(10)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            shutil.rmtree(hb_dir, ignore_errors=True)
            print(f"[launch] attempt {attempt + 1}/{max_restarts + 1} failed: {failed}", file=sys.stderr)
            continue
        shutil.rmtree(hb_dir, ignore_errors=True)
        return 0
    return code if code else 1


def describe_exit(code: Optional[int]) -> str:
    """A rank's exit code in words (75 is ``parallel.comm_guard.EXIT_COMM_FAILURE``)."""
    import signal
    if code is None:
        return "no exit code"
    if code < 0:
        try:
            return f"killed by {signal.Signals(-code).name}"
        except ValueError:
            return f"killed by signal {-code}"
    return {75: "exit 75 (comm watchdog: a hung collective or rank)", 124: "exit 124 (time limit)",
            134: "exit 134 (abort)", 137: "exit 137 (SIGKILL)", 139: "exit 139 (segfault)"}.get(code, f"exit {code}")


def agent_store(timeout_s: float = 60.0):
    """A client of torchrun's agent TCPStore (``TORCHELASTIC_USE_AGENT_STORE=True``: the static and c10d
    rendezvous host it at MASTER_ADDR:MASTER_PORT for the workers' lifetime), or None. Opening it touches
    no GPU."""
    if os.environ.get("TORCHELASTIC_USE_AGENT_STORE") != "True" or "MASTER_PORT" not in os.environ:
        return None
    import datetime

    import torch.distributed as tdist
    try:
        return tdist.TCPStore(os.environ.get("MASTER_ADDR", "127.0.0.1"), int(os.environ["MASTER_PORT"]),
                              is_master=False, timeout=datetime.timedelta(seconds=timeout_s))
    except Exception as e:  # noqa: BLE001 - no store: the caller runs unsupervised
        print(f"[supervise] no agent store ({type(e).__name__}: {e})", file=sys.stderr, flush=True)
        return None


def _die_with_parent() -> None:
    """preexec_fn of a supervised child: SIGKILL when the supervisor dies (Linux PR_SET_PDEATHSIG), so no
    rank process outlives a supervisor that was killed outright."""
    try:
        import ctypes
        import signal
        ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, signal.SIGKILL)  # PR_SET_PDEATHSIG = 1
    except Exception:  # noqa: BLE001 - best effort (non-Linux)
        pass


def _kill_tree(p: "subprocess.Popen", grace_s: float = 10.0) -> None:
    import signal
    for sig, wait in ((signal.SIGTERM, grace_s), (signal.SIGKILL, 30.0)):
        try:
            os.killpg(p.pid, sig)
        except (ProcessLookupError, PermissionError):
            pass
        try:
            p.wait(wait)
            return
        except subprocess.TimeoutExpired:
            continue


def supervise_rank(cmd: List[str], fallback_env: Callable[[str], Dict[str, str]],
                   retryable: Callable[[int], bool], peer_grace_s: float = 30.0,
                   agree_timeout_s: float = 900.0, tag: str = "dbx_supervise") -> int:
    """Run this torchrun rank's work in a CHILD process and, if the attempt fails on any rank, run it
    once more in fresh child processes with ``fallback_env(reason)`` added -- the torchrun form of
    ``run_subprocess_ranks(max_restarts=1)`` for a job that must produce a number (``bench.py`` under the
    driver's ``torch.distributed.run``, whose own ranks cannot be replaced).

    The supervisor never touches the GPU: the child is the process that initialises HIP, so its
    failure (a hung collective ended by the comm watchdog with exit 75, an abort, a segfault) leaves
    the supervisor free to start another. All ranks' supervisors agree through torchrun's agent
    store: each posts its child's exit code; a child still running when a peer has failed gets
    ``peer_grace_s`` to end by itself (its watchdog) before its process group is killed. The retry
    runs only if rank 0's first child did not succeed and some failure is ``retryable``; the retry
    children rendezvous on a fresh port that rank 0 publishes (their own TCPStore, hosted by the
    rank-0 child), so no key of the failed attempt is read again. Returns the last child's exit code.
    """
    import datetime
    rank, world = int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))
    store = agent_store()
    base = dict(os.environ, DBX_SUPERVISED_CHILD="1")
    if store is None:
        return subprocess.run(list(cmd), env=base).returncode

    def key(attempt, what):
        return f"{tag}/{attempt}/{what}"

    def peer_failed(attempt):
        for r in range(world):
            k = key(attempt, f"rc/{r}")
            if r != rank and store.check([k]) and int(store.get(k)) != 0:
                return r
        return None

    def run(attempt, env):
        p = subprocess.Popen(list(cmd), env=env, start_new_session=True, preexec_fn=_die_with_parent)
        current[0] = p
        t_peer = None
        while True:
            try:
                return p.wait(1.0)
            except subprocess.TimeoutExpired:
                pass
            if t_peer is None and peer_failed(attempt) is not None:
                t_peer = time.time()
            if t_peer is not None and time.time() - t_peer > peer_grace_s:
                print(f"[supervise] rank {rank}: a peer failed and this rank's child did not end within "
                      f"{peer_grace_s:.0f}s; killing it", file=sys.stderr, flush=True)
                _kill_tree(p)
                return p.returncode if p.returncode is not None else -9

    # a supervisor that is told to stop (torchrun tearing the group down, a timeout) takes its child's
    # whole process group with it -- the child runs in a session of its own
    current = [None]

    def on_signal(signum, frame):
        if current[0] is not None and current[0].poll() is None:
            _kill_tree(current[0], grace_s=5.0)
        os._exit(128 + signum)
    import signal
    for sig in (signal.SIGTERM, signal.SIGINT, signal.SIGHUP):
        signal.signal(sig, on_signal)

    rc = run(0, base)
    store.set(key(0, f"rc/{rank}"), str(rc))
    keys = [key(0, f"rc/{r}") for r in range(world)]
    try:
        store.wait(keys, datetime.timedelta(seconds=agree_timeout_s))
    except Exception as e:  # noqa: BLE001 - a supervisor that never reported: decide on what is known
        print(f"[supervise] rank {rank}: not every rank reported ({type(e).__name__}); deciding on the "
              f"codes that arrived", file=sys.stderr, flush=True)
    codes = {r: int(store.get(k)) for r, k in enumerate(keys) if store.check([k])}
    bad = {r: c for r, c in sorted(codes.items()) if c != 0}
    if codes.get(0) == 0 or not bad or not any(retryable(c) for c in bad.values()) \
            or any(c in (2, 3) for c in bad.values()):
        return rc
    reason = "attempt 1 failed: " + "; ".join(f"rank {r} {describe_exit(c)}" for r, c in bad.items())
    if rank == 0:
        store.set(key(1, "port"), str(_free_port()))
    port = store.get(key(1, "port")).decode()
    if rank == 0:
        print(f"[supervise] {reason}; re-running every rank once in fresh processes", file=sys.stderr, flush=True)
    env = dict(base, MASTER_PORT=port, TORCHELASTIC_USE_AGENT_STORE="False",
               DBX_RESTART_COUNT=str(int(os.environ.get("DBX_RESTART_COUNT", "0")) + 1))
    env.update(fallback_env(reason))
    rc = run(1, env)
    store.set(key(1, f"rc/{rank}"), str(rc))
    return rc


def main(argv=None) -> int:
    """``python -m dbx_distributed_pytorch_examples_amd.launch --nproc-per-node 8 train.py args...``
    or ``... --nproc-per-node 8 -m package.module args...`` (like torchrun / python -m)."""
    ap = argparse.ArgumentParser(description="dbx launcher (one process per GPU)")
    ap.add_argument("--nproc-per-node", "--nproc_per_node", type=int, default=1)
    ap.add_argument("--nnodes", type=int, default=1)
    ap.add_argument("--node-rank", type=int, default=0)
    ap.add_argument("--master-addr", default="127.0.0.1")
    ap.add_argument("--master-port", type=int, default=0)
    ap.add_argument("--max-restarts", type=int, default=0)
    ap.add_argument("--heartbeat-timeout", type=float, default=0.0)
    ap.add_argument("-m", "--module", action="store_true",
                    help="treat the target as a module name and run it as `python -m <module>`")
    ap.add_argument("script", help="script path (or module name with -m)")
    ap.add_argument("script_args", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    cmd = [sys.executable] + (["-m", a.script] if a.module else [a.script]) + a.script_args
    return run_subprocess_ranks(a.nproc_per_node, cmd, a.nnodes, a.node_rank, a.master_addr,
                                a.master_port or None, a.max_restarts, a.heartbeat_timeout or None)


if __name__ == "__main__":
    sys.exit(main())
