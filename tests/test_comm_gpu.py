"""Framework-owned RCCL communicator (csrc/runtime/comm.cpp, parallel/comm.py): collectives on a
world-1 group on one GPU (exact results), capture inside a HIP graph, and the NativeTrainer's
one-graph step with comm=native bit-identical to the c10d segmented step. Multi-device RCCL
runs only where >= 2 GPUs are visible."""
import copy
import os
import subprocess
import sys

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


@pytest.fixture
def world1(tmp_path):
    if not dist.is_initialized():
        dist.init_process_group("gloo", init_method=f"file://{tmp_path}/pg", rank=0, world_size=1)
    yield
    dist.destroy_process_group()


def test_native_comm_world1_collectives(world1):
    from dbx_distributed_pytorch_examples_amd.parallel.comm import NativeComm, native_comm_available
    assert native_comm_available()
    c = NativeComm()
    x = torch.randn(1000, device="cuda")
    ref = x.clone()
    c.all_reduce(x)
    c.all_reduce(x, op="avg")
    torch.cuda.synchronize()
    assert torch.equal(x, ref)
    out = torch.empty(1000, device="cuda", dtype=torch.bfloat16)
    c.reduce_scatter(out, ref.bfloat16())
    g = torch.empty_like(out)
    c.all_gather(g, out)
    c.broadcast(g)
    torch.cuda.synchronize()
    assert torch.equal(g, ref.bfloat16())
    with pytest.raises(ValueError):
        c.all_gather(torch.empty(3, device="cuda"), torch.empty(2, device="cuda"))
    c.close()


def test_native_comm_captured_in_graph(world1):
    from dbx_distributed_pytorch_examples_amd.parallel.comm import NativeComm
    c = NativeComm()
    x = torch.zeros(4096, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        x.add_(1.0)
        c.all_reduce(x)  # warm RCCL outside capture
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
            x.mul_(2.0)
            c.all_reduce(x)
            x.add_(1.0)
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    assert torch.all(x == 15.0)  # 1 -> 3 -> 7 -> 15
    c.close()


def test_trainer_native_comm_one_graph_matches_segmented(world1, monkeypatch, engine):
    from dbx_distributed_pytorch_examples_amd.engine.native_trainer import NativeTrainer, OptimConfig
    from dbx_distributed_pytorch_examples_amd.models import build_model
    engine(segmented_graphs="1")
    torch.manual_seed(0)
    m1 = build_model("resnet18", num_classes=10)
    m2 = copy.deepcopy(m1)
    engine(comm="native")
    t1 = NativeTrainer(m1, 32, (32, 32), torch.device("cuda"), optim=OptimConfig(lr=0.05))
    engine(comm="torch")
    t2 = NativeTrainer(m2, 32, (32, 32), torch.device("cuda"), optim=OptimConfig(lr=0.05))
    assert t1.ncomm is not None and t2.ncomm is None and t1.segmented and t2.segmented
    g = torch.Generator().manual_seed(1)
    for i in range(6):
        img = torch.randint(0, 256, (32, 32, 32, 3), dtype=torch.uint8, generator=g).cuda()
        lab = torch.randint(0, 10, (32,), generator=g).cuda()
        t1.step(img, lab)
        t2.step(img, lab)
        l1, l2 = t1.read_metrics()[0], t2.read_metrics()[0]
        assert l1 == l2, (i, l1, l2)
    assert len(t1.graphs) == 1 and len(t2.graphs) > 1
    assert torch.equal(t1.prog.master, t2.prog.master)


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs >= 2 GPUs")
def test_native_comm_two_ranks(tmp_path):
    script = tmp_path / "w.py"
    script.write_text(
        "import torch, torch.distributed as dist, os\n"
        "from dbx_distributed_pytorch_examples_amd.parallel.comm import NativeComm\n"
        "r = int(os.environ['RANK']); torch.cuda.set_device(r)\n"
        "dist.init_process_group('gloo')\n"
        "c = NativeComm()\n"
        "x = torch.full((1 << 20,), float(r + 1), device='cuda'); c.all_reduce(x)\n"
        "o = torch.empty(1 << 19, device='cuda'); c.reduce_scatter(o, torch.arange(1 << 20, device='cuda', dtype=torch.float32))\n"
        "torch.cuda.synchronize()\n"
        "assert torch.all(x == 3.0)\n"
        "assert torch.equal(o, 2 * torch.arange(r << 19, (r + 1) << 19, device='cuda', dtype=torch.float32))\n"
        "c.close(); dist.destroy_process_group(); print('OK', r)\n")
    env = dict(os.environ, PYTHONPATH=os.getcwd())
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", "29531", str(script)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.count("OK") == 2


def test_open_verified_comm_world1(world1):
    """The trainer's entry: the communicator passes its check collectives and is returned on every
    rank (here the one rank of a gloo group on one GPU)."""
    from dbx_distributed_pytorch_examples_amd.parallel.comm import open_verified_comm
    c = open_verified_comm(None, torch.device("cuda"))
    assert c is not None and c.verify()


def test_nonblocking_init_and_captured_check(world1):
    """Non-blocking RCCL init (polled to completion), the eager check collectives and the captured one
    (all-reduce on a forked side stream inside a HIP graph, joined back; two replays)."""
    from dbx_distributed_pytorch_examples_amd.parallel.comm import NativeComm
    c = NativeComm(blocking=False, timeout_s=120)
    assert c.async_error()[0] == 0
    assert c.verify(60) and c.verify_captured(60)
    x = torch.arange(1000, device="cuda", dtype=torch.float32)
    c.all_reduce(x)
    torch.cuda.synchronize()
    assert torch.equal(x, torch.arange(1000, device="cuda", dtype=torch.float32))
    c.close()


@pytest.mark.parametrize("comm_side", ["1", "0", "1+defer", "1+defer+lazy", "1+defer+dsf",
                                       "block", "block+btail0", "block+nodefer", "block+nolazy"])
@pytest.mark.parametrize("model,hw,batch", [("resnet18", 32, 32), ("resnet50", 64, 16)])
def test_one_graph_step_post_order_loopback(world1, monkeypatch, model, hw, batch, comm_side, engine):
    """The one-graph multi-rank step's all-reduce ORDER, checked at world 1: with comm_loopback=2
    every bucket all-reduce doubles its range in place (the sum of two identical replicas) and the
    update halves it, so the trajectory equals the plain one bit for bit -- unless a bucket is reduced
    before its weight gradients are final (late posts, batched side stream), which at world 1 with a
    real all-reduce (the identity) would go unnoticed. ``comm_side`` 1: the collectives on the
    weight-gradient side stream behind their batch (event-scoped joins); 0: a separate comm stream
    (both: the batched layout, multirank_layout=batch). "block": the per-block layout of the
    single-GPU step kept in the one-graph step (multirank_layout=block, the default): every segment's
    collective right behind its last block batch, layer1's with the stem's (its last block's tail
    gradients run on the main stream after the stem backward; btail0: none do)."""
    from dbx_distributed_pytorch_examples_amd.engine.native_trainer import NativeTrainer, OptimConfig
    from dbx_distributed_pytorch_examples_amd.models import build_model
    engine(segmented_graphs="1")
    engine(comm="native")
    block = comm_side.startswith("block")
    if block:
        engine(multirank_layout="block")
        if "btail0" in comm_side:
            engine(block_tail_main=0)
        if "nodefer" in comm_side:
            engine(side_defer=0)
        if "nolazy" in comm_side:
            engine(lazy_join=0)
    else:
        engine(multirank_layout="batch")
        engine(comm_side=comm_side[0])
        engine(side_defer="1" if "defer" in comm_side else "0")
        engine(lazy_join="1" if "lazy" in comm_side else "0")
        # "dsf": the downsample forwards on the same side stream as the collectives (ds_fwd_side)
        engine(ds_fwd_side="1" if "dsf" in comm_side else "0")
    torch.manual_seed(0)
    m1 = build_model(model, num_classes=10)
    m2 = copy.deepcopy(m1)
    engine(comm_loopback="2")
    t1 = NativeTrainer(m1, batch, (hw, hw), torch.device("cuda"), optim=OptimConfig(lr=0.05))
    engine(comm_loopback=None)
    t2 = NativeTrainer(m2, batch, (hw, hw), torch.device("cuda"), optim=OptimConfig(lr=0.05))
    assert t1.ncomm is not None and t1.loopback == 2 and t2.loopback == 1
    if block:
        assert t1.block_posts and t1.prog.side_block and not t1.late_posts and t1.comm_side
        assert t1.prog.side_defer == ("nodefer" not in comm_side) and t1.prog.lazy_join == ("nolazy" not in comm_side)
    else:
        assert t1.late_posts and not t1.block_posts
        assert t1.comm_side == (comm_side[0] == "1") and t1.prog.event_joins == t1.comm_side
        assert t1.prog.side_defer == ("defer" in comm_side) and t1.prog.ds_fwd_side == ("dsf" in comm_side)
    g = torch.Generator().manual_seed(1)
    for i in range(6):
        img = torch.randint(0, 256, (batch, hw, hw, 3), dtype=torch.uint8, generator=g).cuda()
        lab = torch.randint(0, 10, (batch,), generator=g).cuda()
        t1.step(img, lab)
        t2.step(img, lab)
        assert t1.read_metrics()[0] == t2.read_metrics()[0], i
    assert len(t1.graphs) == 1
    assert torch.equal(t1.prog.master, t2.prog.master)
