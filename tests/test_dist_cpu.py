"""Multi-process tests on CPU/gloo (world size 2): launcher, failure handling, DDP, ZeRO, the
native program's bucketed all-reduce, and the reference-style frontends."""
import os
import tempfile

import pytest
import torch
import torch.nn as nn

from dbx_distributed_pytorch_examples_amd.launch import Launcher, LaunchError, TorchDistributor

pytestmark = pytest.mark.timeout(600)


def _env_fn(x):
    return {"rank": int(os.environ["RANK"]), "world": int(os.environ["WORLD_SIZE"]), "x": x}


def test_launcher_returns_rank0_result():
    r = TorchDistributor(num_processes=2, local_mode=True, use_gpu=False).run(_env_fn, 7)
    assert r == {"rank": 0, "world": 2, "x": 7}


def _fail_rank1():
    if os.environ["RANK"] == "1":
        raise ValueError("boom from rank 1")
    import time
    time.sleep(30)


def test_launcher_propagates_errors_fast():
    import time
    t = time.time()
    with pytest.raises(LaunchError, match="boom from rank 1"):
        Launcher(2, use_gpu=False).run(_fail_rank1)
    assert time.time() - t < 25  # rank 0 was killed, not waited for


def _faulty_steps(marker_dir):
    from dbx_distributed_pytorch_examples_amd.utils import fault
    for step in range(5):
        fault.heartbeat(step)
        fault.maybe_inject(step)
    with open(os.path.join(marker_dir, f"done{os.environ['RANK']}_{os.environ['DBX_RESTART_COUNT']}"), "w"):
        pass
    return int(os.environ["DBX_RESTART_COUNT"])


def test_fault_injection_and_restart(monkeypatch):
    d = tempfile.mkdtemp()
    monkeypatch.setenv("DBX_FAULT", "1:2:exit")
    r = Launcher(2, use_gpu=False, max_restarts=1).run(_faulty_steps, d)
    assert r == 1  # second attempt succeeded
    assert os.path.exists(os.path.join(d, "done0_1")) and os.path.exists(os.path.join(d, "done1_1"))


def test_watchdog_kills_hung_rank(monkeypatch):
    monkeypatch.setenv("DBX_FAULT", "0:1:hang")
    with pytest.raises(LaunchError, match="watchdog"):
        Launcher(2, use_gpu=False, heartbeat_timeout=3).run(_faulty_steps, tempfile.mkdtemp())


# ---------------------------------------------------------------------------------------------
class TinyNet(nn.Module):
    def __init__(self):
        super().__init__()
        self.c = nn.Conv2d(3, 8, 3, padding=1)
        self.f = nn.Linear(8 * 8 * 8, 5)

    def forward(self, x):
        return self.f(torch.relu(self.c(x)).flatten(1))


def _data(seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(8, 3, 8, 8, generator=g), torch.randint(0, 5, (8,), generator=g)


def _ddp_grads():
    from dbx_distributed_pytorch_examples_amd.parallel import dist as ddist
    from dbx_distributed_pytorch_examples_amd.parallel.ddp import DistributedDataParallel
    ddist.init_distributed(device="cpu")
    torch.manual_seed(0)
    m = DistributedDataParallel(TinyNet(), bucket_cap_mb=0.001)  # tiny buckets: several all-reduces
    x, y = _data()
    r = ddist.get_rank()
    xs, ys = x[r * 4:(r + 1) * 4], y[r * 4:(r + 1) * 4]
    nn.functional.cross_entropy(m(xs), ys).backward()
    m.finish_gradient_sync()
    out = {n: p.grad.clone() for n, p in m.module.named_parameters()}
    ddist.destroy()
    return out, len(m.buckets)


def test_ddp_matches_single_process():
    grads, nb = Launcher(2, use_gpu=False).run(_ddp_grads)
    assert nb > 1
    torch.manual_seed(0)
    ref = TinyNet()
    x, y = _data()
    nn.functional.cross_entropy(ref(x), y).backward()
    for n, p in ref.named_parameters():
        assert torch.allclose(grads[n], p.grad, atol=1e-6, rtol=1e-5), n


def _zero_run(stage):
    from dbx_distributed_pytorch_examples_amd.config import OptimizerConfig
    from dbx_distributed_pytorch_examples_amd.parallel import dist as ddist
    from dbx_distributed_pytorch_examples_amd.parallel.zero import ZeroShardedOptimizer
    ddist.init_distributed(device="cpu")
    torch.manual_seed(0)
    n = 1000
    master = torch.randn(n)
    o = OptimizerConfig(name="adamw", lr=1e-2, weight_decay=0.01)
    z = ZeroShardedOptimizer(master, torch.zeros(n), o, stage=stage)
    r = ddist.get_rank()
    for step in range(3):
        z.grad.copy_(torch.randn(n, generator=torch.Generator().manual_seed(100 * step + r)))
        z.step(grads_already_reduced=False)
    out = master.clone()
    ddist.destroy()
    return out, z.m.numel()


@pytest.mark.parametrize("stage", [1, 2])
def test_zero_matches_plain_optimizer(stage):
    master, shard = Launcher(2, use_gpu=False).run(_zero_run, stage)
    assert shard == 512  # state is sharded
    torch.manual_seed(0)
    p = nn.Parameter(torch.randn(1000))
    opt = torch.optim.AdamW([p], lr=1e-2, weight_decay=0.01)
    for step in range(3):
        g0 = torch.randn(1000, generator=torch.Generator().manual_seed(100 * step))
        g1 = torch.randn(1000, generator=torch.Generator().manual_seed(100 * step + 1))
        p.grad = (g0 + g1) / 2
        opt.step()
    assert torch.allclose(master, p.detach(), atol=1e-5), (master - p.detach()).abs().max()


def _native_dist():
    from dbx_distributed_pytorch_examples_amd.engine.native_trainer import NativeTrainer, OptimConfig
    from dbx_distributed_pytorch_examples_amd.models import build_model
    from dbx_distributed_pytorch_examples_amd.parallel import dist as ddist
    ddist.init_distributed(device="cpu")
    torch.manual_seed(0)
    tr = NativeTrainer(build_model("resnet18", num_classes=4), 4, (32, 32), torch.device("cpu"),
                       optim=OptimConfig(lr=0.0, momentum=0.0, weight_decay=0.0), use_graphs=False,
                       bucket_cap_mb=1.0)
    g = torch.Generator().manual_seed(10 + ddist.get_rank())
    tr.step(torch.randint(0, 256, (4, 32, 32, 3), dtype=torch.uint8, generator=g),
            torch.randint(0, 4, (4,), generator=g))
    out = (tr.prog.grad.clone(), tr.prog.master.clone())
    ddist.destroy()
    return out


@pytest.mark.parametrize("seg_groups", ["", "3:3", "2:4"])
def test_native_program_bucket_allreduce(seg_groups, monkeypatch, engine):
    """world-2 native step (CPU reference ops): grads are summed over ranks in every segment bucket,
    with one all-reduce cut per backward segment (default) or merged segments (seg_groups)."""
    engine(seg_groups=seg_groups)
    g2, m2 = Launcher(2, use_gpu=False).run(_native_dist)
    from dbx_distributed_pytorch_examples_amd.engine.native_trainer import NativeTrainer, OptimConfig
    from dbx_distributed_pytorch_examples_amd.models import build_model
    gs = []
    for r in range(2):
        torch.manual_seed(0)
        tr = NativeTrainer(build_model("resnet18", num_classes=4), 4, (32, 32), torch.device("cpu"),
                           optim=OptimConfig(lr=0.0, momentum=0.0, weight_decay=0.0), use_graphs=False)
        g = torch.Generator().manual_seed(10 + r)
        tr.step(torch.randint(0, 256, (4, 32, 32, 3), dtype=torch.uint8, generator=g),
                torch.randint(0, 4, (4,), generator=g))
        gs.append(tr.prog.grad.clone())
    assert torch.allclose(g2, gs[0] + gs[1], atol=1e-3, rtol=1e-3)


def _mnist_main(d):
    from dbx_distributed_pytorch_examples_amd.frontends import torch_distributor as td
    os.environ["DBX_MLRUNS"] = os.path.join(d, "mlruns")
    return td.main_fn(d, epochs=1)


def test_mnist_main_fn_two_ranks():
    d = tempfile.mkdtemp()
    r = TorchDistributor(num_processes=2, local_mode=True, use_gpu=False).run(_mnist_main, d)
    assert r == "finished"
    assert os.path.exists(os.path.join(d, "checkpoint-1.pth.tar"))
    st = torch.load(os.path.join(d, "checkpoint-1.pth.tar"), weights_only=True)
    assert set(st["model"]) == {"conv1.weight", "conv1.bias", "conv2.weight", "conv2.bias", "fc1.weight", "fc1.bias",
                                "fc2.weight", "fc2.bias"}


def _ray_loop(config):
    from dbx_distributed_pytorch_examples_amd.frontends import ray as rt
    from dbx_distributed_pytorch_examples_amd.utils.checkpoint import save_ray_checkpoint
    m = rt.prepare_model(TinyNet())
    opt = torch.optim.Adam(m.parameters(), lr=config["lr"])
    x, y = _data(rt.get_context().get_world_rank())
    for epoch in range(2):
        loss = nn.functional.cross_entropy(m(x), y)
        opt.zero_grad()
        loss.backward()
        if hasattr(m, "finish_gradient_sync"):
            m.finish_gradient_sync()
        opt.step()
        d = tempfile.mkdtemp()
        save_ray_checkpoint(d, m)
        rt.report({"loss": loss.item(), "epoch": epoch}, checkpoint=rt.Checkpoint.from_directory(d))


def test_ray_style_trainer():
    from dbx_distributed_pytorch_examples_amd.frontends import ray as rt
    store = tempfile.mkdtemp()
    res = rt.TorchTrainer(_ray_loop, train_loop_config={"lr": 1e-2},
                          scaling_config=rt.ScalingConfig(num_workers=2, use_gpu=False),
                          run_config=rt.RunConfig(storage_path=store, name="t")).fit()
    assert res.error is None, res.error
    assert res.metrics["epoch"] == 1.0 and len(res.metrics_history) == 2
    with res.checkpoint.as_directory() as d:
        sd = torch.load(os.path.join(d, "model.pt"), weights_only=True)
    assert "c.weight" in sd


def _accel():
    from dbx_distributed_pytorch_examples_amd.frontends.accelerate import Accelerator
    acc = Accelerator(cpu=True)
    torch.manual_seed(0)
    model = TinyNet()
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    model, opt = acc.prepare(model, opt)
    x, y = _data(acc.process_index)
    loss = nn.functional.cross_entropy(model(x), y)
    acc.backward(loss)
    opt.step()
    g = acc.gather(torch.tensor(float(acc.process_index)))
    s = acc.reduce(torch.tensor(1.0))
    return g.tolist(), float(s), [p.detach().clone() for p in acc.unwrap_model(model).parameters()]


def test_accelerate_style_two_ranks():
    g, s, params = Launcher(2, use_gpu=False).run(_accel)
    assert g == [0.0, 1.0] and s == 2.0


def _divergence_check():
    from dbx_distributed_pytorch_examples_amd.parallel import dist as ddist
    from dbx_distributed_pytorch_examples_amd.parallel.ddp import DistributedDataParallel
    from dbx_distributed_pytorch_examples_amd.utils import debug
    ddist.init_distributed(device="cpu")
    torch.manual_seed(0)
    m = DistributedDataParallel(TinyNet(), bucket_cap_mb=0.001)
    x, y = _data(ddist.get_rank())
    nn.functional.cross_entropy(m(x), y).backward()
    m.finish_gradient_sync()
    debug.check_bucket_order(m.bucket_log)
    debug.assert_replicas_in_sync([p.grad for p in m.module.parameters()], what="grads")  # synced: ok
    caught = False
    if ddist.get_rank() == 1:
        with torch.no_grad():
            next(m.module.parameters()).add_(1e-3)  # rank 1 drifts
    try:
        debug.assert_replicas_in_sync(list(m.module.parameters()))
    except AssertionError:
        caught = True
    ddist.destroy()
    return caught, len(m.bucket_log)


def test_replica_divergence_and_bucket_order_checks():
    caught, nb = Launcher(2, use_gpu=False).run(_divergence_check)
    assert caught and nb > 1


def _two_node_fn():
    import torch.distributed as tdist
    from dbx_distributed_pytorch_examples_amd.parallel import dist as ddist
    ddist.init_distributed(device="cpu")
    t = torch.tensor([float(tdist.get_rank() + 1)])
    tdist.all_reduce(t)
    out = (tdist.get_rank(), tdist.get_world_size(), int(os.environ["GROUP_RANK"]), int(os.environ["LOCAL_RANK"]),
           float(t))
    ddist.destroy()
    return out


def test_two_node_rendezvous_on_one_host():
    """Multi-node plumbing without a cluster: two launchers with nnodes=2 and
    node_rank 0/1 rendezvous on one MASTER_ADDR:PORT and form one 4-rank gloo group."""
    import threading
    from dbx_distributed_pytorch_examples_amd.launch import _free_port
    port = _free_port()
    res = {}

    def node(rank):
        res[rank] = Launcher(2, nnodes=2, node_rank=rank, master_port=port, use_gpu=False, timeout=120).run(_two_node_fn)
    th = threading.Thread(target=node, args=(1,))
    th.start()
    node(0)
    th.join(150)
    assert res[0] == (0, 4, 0, 0, 10.0)
    assert res[1] == (2, 4, 1, 0, 10.0)   # node 1's local rank 0 is global rank 2


def _accel_native():
    """Accelerate-style loop on engine.native_module at world 2 (CPU reference ops, gloo): prepare()
    passes the module through, its backward averages the flat gradient in one collective."""
    import torch.distributed as tdist
    from dbx_distributed_pytorch_examples_amd.engine.native_module import NativeResNet, native_module
    from dbx_distributed_pytorch_examples_amd.frontends.accelerate import Accelerator
    from dbx_distributed_pytorch_examples_amd.models import build_model
    acc = Accelerator(cpu=True)
    torch.manual_seed(0)
    nm = native_module(build_model("resnet18", num_classes=10), 4, (32, 32), torch.device("cpu")).train()
    opt = torch.optim.SGD(nm.parameters(), lr=0.05)
    model, opt = acc.prepare(nm, opt)
    g = torch.Generator().manual_seed(10 + acc.process_index)  # different data per rank
    x, y = torch.randn(4, 3, 32, 32, generator=g), torch.randint(0, 10, (4,), generator=g)
    loss = nn.functional.cross_entropy(model(x), y)
    acc.backward(loss)
    grad = torch.cat([p.grad.reshape(-1) for p in model.parameters()])
    opt.step()
    par = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
    both = [torch.empty_like(grad) for _ in range(2)]
    tdist.all_gather(both, grad)
    pboth = [torch.empty_like(par) for _ in range(2)]
    tdist.all_gather(pboth, par)
    return (isinstance(model, NativeResNet), torch.equal(both[0], both[1]), torch.equal(pboth[0], pboth[1]),
            float(grad.norm()))


def test_accelerate_native_module_two_ranks():
    is_native, grads_equal, params_equal, gnorm = Launcher(2, use_gpu=False).run(_accel_native)
    assert is_native and grads_equal and params_equal and gnorm > 0  # averaged gradients, replicas in sync


def _native_module_sync():
    """engine.native_module at world 2 (gloo, CPU reference ops): rank 0's weights are broadcast at
    construction, the overlapped per-segment all-reduce gives exactly the mean of the per-rank
    single-process gradients, and a short final batch (torch-module fallback) still averages the
    gradients, so the replicas stay identical."""
    import torch.distributed as tdist
    from dbx_distributed_pytorch_examples_amd.engine.native_module import native_module
    from dbx_distributed_pytorch_examples_amd.models import build_model
    from dbx_distributed_pytorch_examples_amd.parallel import dist as ddist
    info = ddist.init_distributed(device="cpu")
    rank = info.rank
    torch.manual_seed(100 + rank)  # different init per rank: the constructor broadcast must fix it
    nm = native_module(build_model("resnet18", num_classes=10), 4, (32, 32), torch.device("cpu")).train()

    def flat(ts):
        return torch.cat([t.detach().reshape(-1) for t in ts])

    def gather(t):
        out = [torch.empty_like(t) for _ in range(2)]
        tdist.all_gather(out, t)
        return out

    par = gather(flat(nm.parameters()))
    init_same = torch.equal(par[0], par[1])
    singles = [tdist.new_group([r]) for r in range(2)]
    ref = build_model("resnet18", num_classes=10)
    ref.load_state_dict(nm.state_dict())
    nm1 = native_module(ref, 4, (32, 32), torch.device("cpu"), process_group=singles[rank]).train()
    g = torch.Generator().manual_seed(10 + rank)
    x, y = torch.randn(4, 3, 32, 32, generator=g), torch.randint(0, 10, (4,), generator=g)
    nn.functional.cross_entropy(nm1(x), y).backward()
    gl = gather(flat(p.grad for p in nm1.parameters()))
    expect = (gl[0] + gl[1]) / 2
    nn.functional.cross_entropy(nm(x), y).backward()
    got = flat(p.grad for p in nm.parameters())
    grad_is_mean = torch.equal(got, expect)
    for p in nm.parameters():
        p.grad = None
    nn.functional.cross_entropy(nm(x[:3]), y[:3]).backward()  # short batch -> torch fallback path
    gs = gather(flat(p.grad for p in nm.parameters()))
    short_synced = torch.equal(gs[0], gs[1]) and float(gs[0].norm()) > 0
    ddist.destroy()
    return init_same, grad_is_mean, short_synced


def test_native_module_broadcast_overlap_and_short_batch_two_ranks():
    init_same, grad_is_mean, short_synced = Launcher(2, use_gpu=False).run(_native_module_sync)
    assert init_same, "rank 0's parameters were not broadcast at construction"
    assert grad_is_mean, "overlapped per-segment all-reduce != mean of per-rank gradients"
    assert short_synced, "short-batch fallback left the replicas' gradients different"


def _native_zero_vs_dp(optim, clip):
    """NativeTrainer ZeRO-1 (per-segment reduce-scatter, sharded update, bf16 all-gather + exact fp32 BN
    exchange) against plain data parallel: the full fp32 parameters after 3 steps must be identical."""
    from dbx_distributed_pytorch_examples_amd.engine.native_trainer import NativeTrainer, OptimConfig
    from dbx_distributed_pytorch_examples_amd.models import build_model
    from dbx_distributed_pytorch_examples_amd.parallel import dist as ddist
    info = ddist.init_distributed(device="cpu")
    from dbx_distributed_pytorch_examples_amd.train.native_step import zero_bytes_label
    out, nbytes, shard = {}, 0, 0
    for z in (0, 1):
        torch.manual_seed(0)
        m = build_model("resnet18", num_classes=10)
        o = OptimConfig(lr=0.05, grad_clip=clip) if optim == "sgd" else \
            OptimConfig(name="adamw", lr=1e-3, weight_decay=0.01, grad_clip=clip)
        tr = NativeTrainer(m, 4, (32, 32), torch.device("cpu"), optim=o, zero_stage=z)
        g = torch.Generator().manual_seed(7 + info.rank)
        for _ in range(3):
            tr.step(torch.randint(0, 256, (4, 32, 32, 3), dtype=torch.uint8, generator=g),
                    torch.randint(0, 10, (4,), generator=g))
        tr.sync_master()
        out[z] = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
        if z:
            nbytes, shard, coll = tr.zero.bytes_per_step, tr.zero.m.numel(), tr.zero.coll
            label = zero_bytes_label(tr.zero)
            assert f"at world {info.world_size}" in label
            if info.world_size < 8:  # a small world still states the 8-rank exchange it plans
                assert "planned at 8 ranks" in label and tr.zero.planned_bytes(8) > 0
    ddist.destroy()
    rel = ((out[0] - out[1]).norm() / out[0].norm()).item()
    return torch.equal(out[0], out[1]), rel, nbytes, shard, out[0].numel(), coll


@pytest.mark.parametrize("world,optim,clip", [(1, "adamw", 0.3), (2, "sgd", 0.0), (2, "adamw", 0.3),
                                              (4, "adamw", 0.0)])
def test_native_zero1_matches_dp(world, optim, clip):
    # world 1: a one-rank process group with the segmented multi-rank path forced (the one-GPU
    # rehearsal configuration): the reduce-scatter / all-gather exchange runs as identities
    env = {"DBX_FORCE_PG": "1", "DBX_ENGINE": "segmented_graphs=1"} if world == 1 else None
    equal, rel, nbytes, shard, n, coll = Launcher(world, use_gpu=False, env=env).run(_native_zero_vs_dp, optim, clip)
    assert coll
    if world <= 2:  # a two-term fp32 sum does not depend on the collective's reduction order
        assert equal, f"ZeRO-1 parameters differ from data parallel (rel {rel})"
    else:  # reduce-scatter vs all-reduce may sum the 4 ranks in another order: last-bit differences
        assert rel < 1e-6, rel
    assert shard <= n // world + 16 * world * 6  # optimizer state is sharded
    # reduce-scatter fp32 + all-gather bf16: ~ (w-1)/w * 6 bytes per parameter (DDP all-reduce alone: 8)
    assert nbytes < (world - 1) / world * 6.2 * n or world == 1


def _comm_hang_train(ckpt_dir):
    """train() with checkpoints; rank 1 stops issuing collectives at step 3 (epoch 2) on the first
    attempt. The comm watchdog (or the bounded c10d timeout) must end rank 0, the launcher restarts
    the job, and the second attempt resumes from the epoch-1 checkpoint."""
    from dbx_distributed_pytorch_examples_amd.config import TrainConfig
    from dbx_distributed_pytorch_examples_amd.data.datasets import SyntheticImages
    from dbx_distributed_pytorch_examples_amd.train.engine import train
    cfg = TrainConfig(model="tiny", num_classes=5, batch_size=4, epochs=2, log_every=0, checkpoint_dir=ckpt_dir,
                      engine="autograd")
    cfg.optim.lr = 0.01
    cfg.data.num_workers = 0
    torch.manual_seed(0)
    res = train(cfg, model=TinyNet(), train_dataset=SyntheticImages(16, 8, 3, 5, seed=1,
                                                                     transform=_to_tensor), log_mlflow=False)
    return int(os.environ["DBX_RESTART_COUNT"]), res.resumed_epoch, res.steps, len(res.history)


def _to_tensor(img):
    import numpy as np
    return torch.from_numpy(np.array(img)).permute(2, 0, 1).float() / 255


def test_comm_hang_is_aborted_and_job_resumes(tmp_path):
    import time
    t = time.time()
    out = Launcher(2, use_gpu=False, max_restarts=1, heartbeat_timeout=120,
                   env={"DBX_FAULT": "1:3:comm_hang", "DBX_COMM_TIMEOUT": "5"}).run(
        _comm_hang_train, str(tmp_path))
    restarts, resumed_epoch, steps, hist = out
    assert restarts == 1 and resumed_epoch == 1 and steps == 4 and hist == 2, out
    assert time.time() - t < 90  # detected within the 5 s bound, not the 30 min default


def test_comm_watchdog_unit():
    """CommWatchdog.check: an RCCL async error or an over-age step is reported; fire() aborts the
    communicators and exits with EXIT_COMM_FAILURE."""
    from dbx_distributed_pytorch_examples_amd.parallel.comm_guard import EXIT_COMM_FAILURE, CommWatchdog

    class FakeComm:
        def __init__(self):
            self.code, self.aborted = 0, False

        def async_error(self):
            return self.code, "remote process exited" if self.code else ""

        def abort(self):
            self.aborted = True
    exits = []
    c = FakeComm()
    wd = CommWatchdog(timeout_s=0.3, poll_s=0.05, comms=[c], exit_fn=exits.append)
    wd.step_begin(0)
    wd.step_end()
    assert wd.check() is None
    c.code = 6  # ncclRemoteError
    import time
    for _ in range(100):
        if exits:
            break
        time.sleep(0.05)
    assert exits == [EXIT_COMM_FAILURE] and c.aborted and "async error 6" in wd.fired
    wd2 = CommWatchdog(timeout_s=0.2, poll_s=10, comms=[], exit_fn=exits.append)
    wd2.step_begin(7)
    time.sleep(0.3)
    assert "step 7" in wd2.check()
    wd.close()
    wd2.close()


def test_open_verified_comm_falls_back_together(tmp_path):
    """Without RCCL (CPU / gloo) every rank gets None from open_verified_comm -- the agreed c10d
    fallback -- with a warning, instead of some ranks taking the framework-communicator path."""
    import warnings
    import torch.distributed as tdist
    from dbx_distributed_pytorch_examples_amd.parallel.comm import open_verified_comm
    tdist.init_process_group("gloo", init_method=f"file://{tmp_path}/pg", rank=0, world_size=1)
    try:
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter("always")
            assert open_verified_comm(None, torch.device("cpu")) is None
        assert any("c10d" in str(x.message) for x in w)
    finally:
        tdist.destroy_process_group()


def test_watchdog_closed_when_a_step_raises(tmp_path):
    """A step that raises inside train() must not leave the comm watchdog armed: a caller that catches
    the exception and carries on (a notebook, an in-process retry) would otherwise be killed
    DBX_COMM_TIMEOUT seconds later by the watchdog's exit."""
    import subprocess
    import sys
    script = tmp_path / "w.py"
    script.write_text(
        "import sys, time, torch\n"
        f"sys.path.insert(0, {os.path.dirname(os.path.abspath(__file__))!r})\n"
        "from test_dist_cpu import TinyNet, _to_tensor\n"
        "from dbx_distributed_pytorch_examples_amd.config import TrainConfig\n"
        "from dbx_distributed_pytorch_examples_amd.data.datasets import SyntheticImages\n"
        "from dbx_distributed_pytorch_examples_amd.train.engine import train\n"
        "cfg = TrainConfig(model='tiny', num_classes=5, batch_size=4, epochs=1, log_every=0, engine='autograd')\n"
        "cfg.data.num_workers = 0\n"
        "class Boom(TinyNet):\n"
        "    calls = 0\n"
        "    def forward(self, x):\n"
        "        Boom.calls += 1\n"
        "        if Boom.calls == 2:\n"
        "            raise RuntimeError('injected fault inside the step')\n"
        "        return super().forward(x)\n"
        "try:\n"
        "    train(cfg, model=Boom(), train_dataset=SyntheticImages(16, 8, 3, 5, seed=1, transform=_to_tensor),\n"
        "          log_mlflow=False)\n"
        "except RuntimeError as e:\n"
        "    print('caught', e, flush=True)\n"
        "time.sleep(4)\n"
        "print('alive', flush=True)\n")
    env = dict(os.environ, DBX_COMM_TIMEOUT="1",
               PYTHONPATH=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    r = subprocess.run([sys.executable, str(script)], env=env, capture_output=True, text=True, timeout=300)
    assert "caught injected fault" in r.stdout, r.stderr[-2000:]
    assert r.returncode == 0 and "alive" in r.stdout, (r.returncode, r.stderr[-2000:])
