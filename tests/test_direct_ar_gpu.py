"""Direct two-shot all-reduce kernel (csrc/direct_ar.hip) on one GPU: W "ranks" are W buffers of one
process meeting at the flag barriers through the same peer-pointer protocol the multi-GPU path
uses (there, the pointers are hipIPC mappings of the peers' buffers). The protocol tests run every
rank's workgroups in ONE dispatch (``dar_launch_multi``: co-resident by construction, W up to 8);
the per-rank launch path (``dar_launch``, one kernel per rank) runs two ranks on a normal and a
high-priority stream (two hardware queues). Results must equal the fp32 rank-order sum bit for bit
on every rank, across repeated calls (generation counters) and graph replays; a missing peer ends
the kernel at its deadline with the error bit set instead of hanging the device."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _C():
    from dbx_distributed_pytorch_examples_amd.ops._ext import C
    return C()


def _launch(c, bufs, fl, n, grid, timeout, streams, ranks=None):
    world = len(bufs)
    for r in (range(world) if ranks is None else ranks):
        c.dar_launch([b.data_ptr() for b in bufs], [f[0] for f in fl], fl[r][1], fl[r][2], n, r, world, grid,
                     timeout, streams[r].cuda_stream, fl[r][4])


def _ref(src):
    ref = src[0].clone()
    for s in src[1:]:
        ref = ref + s  # fp32, rank order: what the segment owner computes
    return ref


@pytest.mark.parametrize("world,n", [(2, 1 << 20), (3, 100003), (8, 1 << 18), (5, 7), (4, 1), (1, 4099)])
def test_direct_two_shot_protocol(world, n):
    c = _C()
    grid = 8
    torch.manual_seed(world * 7 + n)
    src = [torch.randn(n, device="cuda") for _ in range(world)]
    ref = _ref(src)
    bufs = [s.clone() for s in src]
    fl = [c.dar_alloc(grid) for _ in range(world)]
    try:
        for _ in range(3):  # repeated calls: the per-workgroup generations advance in step
            for b, s in zip(bufs, src):
                b.copy_(s)
            c.dar_launch_multi([b.data_ptr() for b in bufs], [f[0] for f in fl], [f[1] for f in fl],
                               [f[2] for f in fl], n, grid, 20.0, torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            assert [c.dar_read_err(f[2]) for f in fl] == [0] * world
            for b in bufs:
                assert torch.equal(b, ref)
    finally:
        for f in fl:
            c.dar_free(*f[:4])


def test_direct_per_rank_launches_on_two_queues():
    """The production launch (one kernel per rank) with the two ranks on a normal- and a
    high-priority stream, so they land on different hardware queues and run side by side."""
    c = _C()
    world, grid, n = 2, 8, 1 << 20
    src = [torch.randn(n, device="cuda") for _ in range(world)]
    ref = _ref(src)
    bufs = [s.clone() for s in src]
    fl = [c.dar_alloc(grid) for _ in range(world)]
    streams = [torch.cuda.Stream(priority=0), torch.cuda.Stream(priority=-1)]
    try:
        for _ in range(2):
            for b, s in zip(bufs, src):
                b.copy_(s)
            torch.cuda.synchronize()
            _launch(c, bufs, fl, n, grid, 20.0, streams)
            torch.cuda.synchronize()
            assert [c.dar_read_err(f[2]) for f in fl] == [0] * world
            for b in bufs:
                assert torch.equal(b, ref)
    finally:
        for f in fl:
            c.dar_free(*f[:4])


def test_direct_two_shot_graph_replay():
    c = _C()
    world, grid, n = 4, 8, 65536 + 12
    src = [torch.randn(n, device="cuda") for _ in range(world)]
    ref = _ref(src)
    bufs = [s.clone() for s in src]
    fl = [c.dar_alloc(grid) for _ in range(world)]
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    try:
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                c.dar_launch_multi([b.data_ptr() for b in bufs], [f[0] for f in fl], [f[1] for f in fl],
                                   [f[2] for f in fl], n, grid, 20.0, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        for _ in range(3):  # the generations advance on the device: every replay meets its peers
            for b, x in zip(bufs, src):
                b.copy_(x)
            g.replay()
            torch.cuda.synchronize()
            assert [c.dar_read_err(f[2]) for f in fl] == [0] * world
            for b in bufs:
                assert torch.equal(b, ref)
    finally:
        del g
        torch.cuda.synchronize()
        for f in fl:
            c.dar_free(*f[:4])


def test_direct_missing_peer_times_out_with_error_bit():
    c = _C()
    world, grid, n = 2, 4, 4096
    bufs = [torch.ones(n, device="cuda") for _ in range(world)]
    fl = [c.dar_alloc(grid) for _ in range(world)]
    streams = [torch.cuda.Stream() for _ in range(world)]
    try:
        assert c.dar_host_err(fl[0][3]) == 0
        _launch(c, bufs, fl, n, grid, 0.2, streams, ranks=[0])  # rank 1 never arrives
        torch.cuda.synchronize()  # bounded: the first barrier gives up at its deadline, no later waits
        assert c.dar_host_err(fl[0][3]) == 1  # the pinned mirror the comm watchdog polls (no device sync)
        assert c.dar_read_err(fl[0][2], True) == 1
        assert c.dar_read_err(fl[0][2]) == 0  # reset
        # the timed-out rank's result is poisoned, never a partial sum passed off as a gradient
        assert torch.isnan(bufs[0]).all() and torch.equal(bufs[1], torch.ones(n, device="cuda"))
    finally:
        for f in fl:
            c.dar_free(*f[:4])


def test_direct_allreduce_class_world1(tmp_path):
    """The registration path (IPC handles of the buffer and the uncached flag array, the agreement)
    on a one-rank group; the kernel reduces over one rank (identity) and verifies."""
    import torch.distributed as dist
    from dbx_distributed_pytorch_examples_amd.parallel.comm import DirectAllReduce, NativeComm
    dist.init_process_group("gloo", init_method=f"file://{tmp_path}/pg", rank=0, world_size=1)
    try:
        nc = NativeComm()
        buf = torch.randn(1 << 18, device="cuda")
        keep = buf.clone()
        d = DirectAllReduce(nc, buf, grid=8)
        assert d.verify(30.0) and torch.equal(buf, keep)
        assert d.in_buffer(buf[16:1024]) and not d.in_buffer(buf[1:1024])  # 16-byte aligned ranges only
        assert not d.in_buffer(torch.empty(16, device="cuda")) and not d.takes(buf[16:1024])  # world 1: RCCL
        d.all_reduce(buf[:4096])
        torch.cuda.synchronize()
        assert torch.equal(buf, keep) and d.errors() == 0
        d.close()
        nc.close()
    finally:
        dist.destroy_process_group()
