"""xGMI-aware collective plan: which path and which bucket size each gradient collective takes.

SURVEY.md §5.8 / §2.5 M3. The reference reaches NCCL only through c10d and DDP's reducer with its
NVSwitch-era defaults (25 MiB buckets; `01_torch_distributor/01_basic_torch_distributor.py:291`)
and touches the transport only through ``NCCL_DEBUG`` (`setup/00_setup.py:122-123`). An MI355X node
is different: no switch, a FULL MESH of point-to-point xGMI links (7 per GPU, ~153 GB/s each per
direction), so

* a ring all-reduce drives only the two links of its ring per channel and pays 2(n-1) dependent
  steps; RCCL spreads many channels (rings) over the 7 links for bandwidth, but the step latency
  stays -- it dominates the small buckets;
* a direct two-shot all-reduce (``csrc/direct_ar.hip``: reduce-scatter by reading 1/n of every
  peer's buffer over its own link, then all-gather the same way) moves the same bytes per link,
  2S/n, in two data steps and three flag barriers -- the better choice up to a size where the
  ring's pipelining wins.

:func:`plan_allreduce` prices both with the model below and returns the plan for one buffer: path
(``rccl`` | ``direct``), the chunking of the buffer into buckets, and the RCCL channel bounds of the
framework communicator. The model's constants are ASSUMPTIONS (link rate from the platform spec,
latencies from the one-GPU flag hand-off measurements in the image's CDNA4 guide,
/opt/skills/guides/MI355X_MICROARCH.md -- outside this repository); the world >= 2
measurement that would calibrate them needs a multi-GPU node (``tools/bench_allreduce.py --path
all`` prints the nccl-tests lines to do so). Until then the direct path is opt-in
(engine field ``direct_ar=1``) and the defaults keep RCCL for everything.

:func:`two_shot_segments` / :func:`two_shot_reference` are the direct kernel's index math in Python
(segments, per-workgroup stripes, the scalar tail), used by the CPU tests.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np

# what csrc/direct_ar.hip compiles for
DAR_MAX_RANKS = 8
DAR_THREADS = 256


@dataclass(frozen=True)
class XgmiTopology:
    """One node of MI355X GPUs on a full xGMI mesh (assumed constants, see the module doc)."""
    world: int
    links_per_gpu: int = 7
    link_gbps: float = 153.0       # per link and direction
    ring_step_us: float = 3.0      # one dependent ring step (RCCL LL/LL128 hop incl. kernel-side sync)
    barrier_us: float = 2.5        # one cross-GPU flag barrier of the direct kernel
    launch_us: float = 4.0         # one collective kernel launch / graph node
    ring_efficiency: float = 0.80  # fraction of the link rate a multi-channel ring sustains
    direct_efficiency: float = 0.70  # ... the direct kernel's remote loads sustain

    @property
    def full_mesh(self) -> bool:
        return self.world <= self.links_per_gpu + 1


def ring_allreduce_us(nbytes: int, topo: XgmiTopology, channels: Optional[int] = None) -> float:
    """Ring all-reduce: 2(n-1) steps; each rank sends 2(n-1)/n of the buffer, spread over the links
    its channels' rings use (one outgoing link per ring; RCCL lays rings over distinct links)."""
    n = topo.world
    if n <= 1:
        return 0.0
    ch = channels or topo.links_per_gpu
    links = min(ch, topo.links_per_gpu)
    per_link = 2.0 * (n - 1) / n * nbytes / links
    bw = topo.link_gbps * 1e3 * topo.ring_efficiency  # bytes per us
    return topo.launch_us + 2 * (n - 1) * topo.ring_step_us + per_link / bw


def direct_allreduce_us(nbytes: int, topo: XgmiTopology) -> float:
    """Direct two-shot: 3 barriers + 2 data steps; each step reads nbytes/n from every peer, each over
    its own link (full mesh), so a link carries nbytes/n per step."""
    n = topo.world
    if n <= 1:
        return 0.0
    if not topo.full_mesh or n > DAR_MAX_RANKS:
        return math.inf
    bw = topo.link_gbps * 1e3 * topo.direct_efficiency
    return topo.launch_us + 3 * topo.barrier_us + 2 * (nbytes / n) / bw


@dataclass
class AllReducePlan:
    path: str                       # "rccl" | "direct"
    buckets: List[Tuple[int, int]]  # [lo, hi) element ranges, issued in order
    est_us: float                   # model estimate for the whole buffer
    min_ctas: int = 0               # RCCL channel bounds of the communicator (0: RCCL's choice)
    max_ctas: int = 0


def _cfg(cfg=None):
    from ..engine_config import EngineConfig
    return cfg or EngineConfig.current()


def direct_enabled(cfg=None) -> bool:
    return _cfg(cfg).direct_ar


def direct_max_bytes(cfg=None) -> int:
    return int(_cfg(cfg).direct_ar_max_mb * (1 << 20))


def rccl_channel_bounds(world: int, cfg=None) -> Tuple[int, int]:
    """RCCL CTA (channel) bounds for the framework communicator (engine fields ``rccl_min_ctas`` /
    ``rccl_max_ctas``; 0 = RCCL's own tuning, the default: the plan's bucket sizes are what the
    framework picks)."""
    c = _cfg(cfg)
    return int(c.rccl_min_ctas), int(c.rccl_max_ctas)


def plan_allreduce(numel: int, elem_bytes: int, world: int, bucket_cap_elems: int,
                   topo: Optional[XgmiTopology] = None, allow_direct: Optional[bool] = None) -> AllReducePlan:
    """Plan one gradient range: RCCL buckets of ``bucket_cap_elems`` (few, large messages -- the
    per-bucket step latency is paid 2(n-1) times), or the direct path for the whole range when it is
    enabled, fits ``direct_ar_max_mb`` and the model prices it below the ring."""
    topo = topo or XgmiTopology(world)
    nbytes = numel * elem_bytes
    allow = direct_enabled() if allow_direct is None else allow_direct
    ring = sum(ring_allreduce_us((hi - lo) * elem_bytes, topo) for lo, hi in chunk(numel, bucket_cap_elems))
    lo_ctas, hi_ctas = rccl_channel_bounds(world)
    if allow and world > 1 and nbytes <= direct_max_bytes():
        d = direct_allreduce_us(nbytes, topo)
        if d < ring:
            return AllReducePlan("direct", [(0, numel)], d, lo_ctas, hi_ctas)
    return AllReducePlan("rccl", chunk(numel, bucket_cap_elems), ring, lo_ctas, hi_ctas)


def chunk(numel: int, cap: int) -> List[Tuple[int, int]]:
    cap = max(1, int(cap))
    return [(lo, min(numel, lo + cap)) for lo in range(0, numel, cap)] or [(0, 0)]


def crossover_bytes(world: int, topo: Optional[XgmiTopology] = None) -> int:
    """The largest power-of-two buffer the model prices faster on the direct path (0: never)."""
    topo = topo or XgmiTopology(world)
    best = 0
    for e in range(10, 34):
        b = 1 << e
        if direct_allreduce_us(b, topo) < ring_allreduce_us(b, topo):
            best = b
    return best


# ---- the direct kernel's index math (csrc/direct_ar.hip), for the CPU tests --------------------
def two_shot_segments(n: int, world: int) -> List[Tuple[int, int]]:
    """Segment r = [r*S, min(n, (r+1)*S)), S = ceil(n / world) rounded up to 4 elements."""
    seg = ((n + world - 1) // world + 3) & ~3
    return [(min(n, r * seg), min(n, (r + 1) * seg)) for r in range(world)]


def stripe_owner(i4: int, grid: int) -> int:
    """The workgroup that owns float4 index ``i4`` of a segment (grid-stride loop of 256 threads)."""
    return (i4 // DAR_THREADS) % grid


def _kernel_float4_visits(n4: int, grid: int):
    """The (workgroup, float4 index) pairs of the kernel's grid-stride loop, in its loop order."""
    stride = grid * DAR_THREADS
    for b in range(grid):
        for tid in range(DAR_THREADS):
            i = b * DAR_THREADS + tid
            while i < n4:
                yield b, i
                i += stride


def two_shot_reference(bufs: Sequence[np.ndarray], grid: int = 8) -> List[np.ndarray]:
    """Emulate the two-shot kernel over ``world`` rank buffers following its loops (reduce-scatter of
    segment r by rank r in rank order, scalar tail by workgroup 0, all-gather from each owner);
    returns every rank's result and checks that each element is written exactly once per rank."""
    world = len(bufs)
    src = [b.astype(np.float32).copy() for b in bufs]
    out = [b.copy() for b in src]
    n = src[0].size
    segs = two_shot_segments(n, world)
    covered = [np.zeros(n, dtype=np.int32) for _ in range(world)]
    for r in range(world):  # reduce-scatter
        lo, hi = segs[r]
        n4 = (hi - lo) >> 2
        for b, i in _kernel_float4_visits(n4, grid):
            assert stripe_owner(i, grid) == b
            sl = slice(lo + 4 * i, lo + 4 * i + 4)
            s = src[0][sl].copy()
            for j in range(1, world):
                s = s + src[j][sl]
            out[r][sl] = s
            covered[r][sl] += 1
        for t in range(lo + 4 * n4, hi):  # scalar tail: workgroup 0, threads 0..3
            assert t - (lo + 4 * n4) < 4
            s = src[0][t]
            for j in range(1, world):
                s = np.float32(s + src[j][t])
            out[r][t] = s
            covered[r][t] += 1
    red = [o.copy() for o in out]
    for r in range(world):  # all-gather
        for jj in range(1, world):
            j = (r + jj) % world
            lo, hi = segs[j]
            out[r][lo:hi] = red[j][lo:hi]
            covered[r][lo:hi] += 1
    if any(not (c == 1).all() for c in covered):
        raise AssertionError("two-shot emulation: an element was not written exactly once")
    return out
