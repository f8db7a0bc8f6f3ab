"""xGMI collective plan (parallel/collective_plan.py): the direct two-shot kernel's index math and the
path / bucket choice. CPU only; the kernel itself: tests/test_direct_ar_gpu.py."""
import numpy as np
import pytest

from dbx_distributed_pytorch_examples_amd.parallel import collective_plan as cp


@pytest.mark.parametrize("n", [1, 3, 4, 17, 1000, 4097, 70001])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_two_shot_emulation_is_the_rank_order_sum_on_every_rank(n, world):
    rng = np.random.default_rng(n * 10 + world)
    bufs = [rng.standard_normal(n).astype(np.float32) for _ in range(world)]
    ref = bufs[0].copy()
    for b in bufs[1:]:
        ref = ref + b  # fp32, rank order: what every segment owner computes
    out = cp.two_shot_reference(bufs, grid=3)
    assert all(np.array_equal(o, ref) for o in out)


@pytest.mark.parametrize("n", [0, 1, 5, 64, 1001, 123457])
@pytest.mark.parametrize("world", [1, 2, 5, 8])
def test_segments_tile_the_buffer_on_16_byte_boundaries(n, world):
    segs = cp.two_shot_segments(n, world)
    assert len(segs) == world
    pos = 0
    for lo, hi in segs:
        assert lo == pos and lo <= hi and lo % 4 == 0 or lo == n
        pos = hi
    assert pos == n
    # only the last non-empty segment may end off a 4-element boundary (the kernel's scalar tail)
    ragged = [i for i, (lo, hi) in enumerate(segs) if (hi - lo) % 4]
    assert len(ragged) <= 1 and all(segs[i][1] == n for i in ragged)


def test_stripes_are_owned_by_one_workgroup():
    grid = 5
    seen = {}
    for b, i in cp._kernel_float4_visits(3 * cp.DAR_THREADS * grid + 17, grid):
        assert i not in seen and cp.stripe_owner(i, grid) == b
        seen[i] = b
    assert len(seen) == 3 * cp.DAR_THREADS * grid + 17


def test_model_prefers_direct_for_small_and_ring_chunks_for_large():
    topo = cp.XgmiTopology(8)
    assert cp.direct_allreduce_us(64 << 10, topo) < cp.ring_allreduce_us(64 << 10, topo)
    assert cp.direct_allreduce_us(1 << 30, topo) > cp.ring_allreduce_us(1 << 30, topo)
    x = cp.crossover_bytes(8)
    assert (1 << 20) <= x < (1 << 30)
    assert cp.direct_allreduce_us(1 << 20, cp.XgmiTopology(16)) == float("inf")  # beyond one mesh
    assert cp.ring_allreduce_us(1 << 20, cp.XgmiTopology(1)) == 0.0


def test_plan_paths(monkeypatch, engine):
    engine(direct_ar=None)
    p = cp.plan_allreduce(1 << 18, 4, 8, 1 << 24)
    assert p.path == "rccl" and p.buckets == [(0, 1 << 18)]  # direct is opt-in
    p = cp.plan_allreduce(1 << 18, 4, 8, 1 << 24, allow_direct=True)
    assert p.path == "direct" and p.buckets == [(0, 1 << 18)]
    engine(direct_ar_max_mb="0.5")
    assert cp.plan_allreduce(1 << 18, 4, 8, 1 << 24, allow_direct=True).path == "rccl"  # 1 MiB > cap
    big = cp.plan_allreduce(25_557_032, 4, 8, 16 << 20)
    assert big.path == "rccl" and big.buckets[0] == (0, 16 << 20) and big.buckets[-1][1] == 25_557_032
    assert cp.plan_allreduce(100, 4, 1, 64, allow_direct=True).path == "rccl"  # world 1: nothing to reduce


def test_channel_bounds_passthrough(monkeypatch, engine):
    engine(rccl_min_ctas=None)
    engine(rccl_max_ctas=None)
    assert cp.rccl_channel_bounds(8) == (0, 0)
    engine(rccl_min_ctas="7")
    assert cp.rccl_channel_bounds(8) == (7, 0)
