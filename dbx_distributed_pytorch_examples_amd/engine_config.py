"""Typed engine configuration: every schedule / kernel / communication switch of the native engine in
one dataclass (one typed config instead of scattered flags).

The reference has one tuning surface, the DeepSpeed dict (`02_deepspeed/deepspeed_config.py:5-50`,
accepted by ``config.from_deepspeed``); the native engine adds the step schedule of the HIP-graph
training step. Each field's default is the measured winner (the profile directory that measured it is
named next to the field); ``None`` means "decided by the step-size policy" -- :class:`StepPolicy`
names the forward-conv-FLOP classes those decisions switch on instead of literal thresholds.

Where the engine reads it: ``EngineConfig.current()`` -- the process default, overridable for A/B runs
through ONE environment variable::

    DBX_ENGINE="side_cu_reserve=64,lazy_join=1,comm=torch"

(``key=value`` pairs, comma separated; booleans 0/1; unknown keys are an error). Code that builds a
program can also pass an ``EngineConfig`` explicitly (``ResNetProgram(..., engine=cfg)``,
``NativeTrainer(..., engine=cfg)``).
"""
from __future__ import annotations

import dataclasses
import os
from dataclasses import dataclass, field, fields
from typing import Optional

ENV = "DBX_ENGINE"


@dataclass(frozen=True)
class StepPolicy:
    """Step-size classes (forward conv FLOPs of one training step) the automatic defaults switch on.
    The three measured presets sit in one class each: ResNet-18 CIFAR-10 b256 (0.02 TFLOP, "tiny"),
    ResNet-50 TinyImageNet b512 (0.35 TFLOP, "small") and the ResNet-50 ImageNet b1024 headline
    (8.4 TFLOP, "large")."""
    tiny_step_flops: float = 5e10    # below: launch-bound CIFAR class
    small_step_flops: float = 5e11   # below: TinyImageNet class (from tiny up); above: headline class

    def tiny(self, flops: float) -> bool:
        return flops < self.tiny_step_flops

    def small(self, flops: float) -> bool:
        return flops < self.small_step_flops

    def mid(self, flops: float) -> bool:  # the TinyImageNet class
        return self.tiny_step_flops <= flops < self.small_step_flops


@dataclass
class EngineConfig:
    # ---- weight-gradient overlap / step schedule (engine/program.py, engine/native_trainer.py) ----
    # side stream for weight gradients: 0 in order, 1 one fork per gradient, 2 one fork per backward
    # segment, 3 one fork per residual block; None: 3 (r5_side_defer/mode3.txt), the multi-rank
    # one-graph step keeps 2 with late collective posts
    overlap_wgrad: Optional[int] = None
    # launch each side batch after the main chain's next kernel (separate hardware queues);
    # None: small steps and the per-block layout (r5_side_defer/)
    side_defer: Optional[bool] = None
    # side-stream weight gradients sized to all but N CUs; None: 128 from the TinyImageNet class up
    # (64 in the multi-rank batched layout), 0 below (r5_cu_reserve/)
    side_cu_reserve: Optional[int] = None
    # no intermediate side-stream joins; None: tiny steps and the per-block layout (r5_side_defer/lazy_join.txt)
    lazy_join: Optional[bool] = None
    # stem weight gradient on the main stream; None: small steps and the per-block layout (r5_tail/)
    stem_wg_main: Optional[bool] = None
    # the last side batch's last N weight gradients on the main stream; None: 3 / 2 (deferred or not)
    # for the TinyImageNet class, else 0 (r5_tail/)
    tail_main: Optional[int] = None
    # per-block layout: the last block's last N weight gradients on the main stream (r5_side_defer/block_tail.txt)
    block_tail_main: int = 2
    # the downsample conv's forward on the side stream beside conv2 / conv3 (r5_side_defer/ds_fwd.txt)
    ds_fwd_side: bool = True
    # the fused conv3 backward's persistent grid spans N CUs (0 = all); None: 128 for the TinyImageNet class
    dwf_cus: Optional[int] = None
    # the optimizer inside the backward: the first N backward segments' SGD / Adam updates (head, layer4,
    # layer3, ...) on the side stream right behind each segment's last block batch (and collective); the
    # rest in one update at the end of the step (-1: every segment, 0: off). Off: measured 1 % slower on
    # ResNet-18 CIFAR and flat on TinyImageNet / the headline for every N (profiles/r6_optbw/)
    overlap_optimizer: int = 0
    # ---- fusion structure ----
    fuse_tail: bool = True          # block outputs computed in the next conv1's prologue
    fuse_bwd_apply: bool = True     # BN-backward apply of a 1x1 conv's output BN in its dgrad prologue
    fuse_dw: bool = True            # bottleneck conv3 backward as one kernel (r2s4_dwfused/)
    fuse_dw_min_tiles: int = 4      # ... where every resident workgroup walks at least N tiles
    fuse_dw_min_hw: int = 0         # ... and only on maps of at least this size (56: layer1 only)
    fuse_stem_bwd: bool = False     # stem backward as one kernel (slower: r2s4_stem/)
    fast_mat: bool = True           # materialised BN output for 3x3 consumers on the eight-wave kernel
    act_writeback: bool = True      # block-internal BN outputs stored by the MASK_Y dgrad epilogue
    pool_reduce: bool = True        # max-pool forward keeps the pooled maxima for the backward
    # which BN-backward applies fold into the next dgrad's prologue; None: 2^25 elements / ratio 1
    # (without the side stream: every one, ratio 8; r3s2_knobs/, r2s3_fold/)
    fold_min_elems: Optional[int] = None
    fold_max_ratio: Optional[float] = None
    fold_ratio_min_hw: int = 56
    # BN finalize in the consumer (forward: consuming conv's prologue; backward: the apply pass) and
    # statistics shards per BN; None: fin_in on for the CIFAR class only (r6_tiny_fin/), coeff_in on and
    # 4 shards for small steps, off with 32 shards above
    # (r4_s6/, r4_s7/, r4_s18/)
    fin_in: Optional[bool] = None
    coeff_in: Optional[bool] = None
    coeff_in_maxc: Optional[int] = None  # None: 512 for the TinyImageNet class, no limit below; 0 = none
    nshard: Optional[int] = None
    # split-K reductions of a side batch deferred to one batched reduce; None: tiny steps (r4_s12/)
    defer_reduce: Optional[bool] = None
    # ---- kernels (ops/kernels.py) ----
    tap_prune: bool = True          # conv launches skip filter taps that only see padding (r3s2_tap_prune/)
    fast: bool = True               # eight-wave kernel entries of the tune table
    conv_dma: int = -1              # force one conv operand path (0-6; -1: per-shape tune table)
    patch3: str = "all"             # weights-stationary 3x3 patch kernels: all | fwd | dgrad | wgrad | none
    patch3_stream: str = "dgrad"    # which patch kernels stream their input
    stem_patch: bool = True         # stem forward on the patch kernel
    stem_wgrad: str = "tile"        # stem weight gradient: tile | generic
    wgrad_rounds: float = 2.0       # split-K depth target of the weight gradients (workgroup rounds)
    wgrad_fuse_max: int = 1 << 20   # largest weight gradient reduced in-launch
    head_splitk: bool = True        # split-K for the few-tile classifier-head GEMMs (r5_headsplit/)
    # split-K of the few-tile forward / data-gradient convs (the small maps of the small steps): a launch
    # of fewer than splitk_wgs tiles splits its K blocks into slices of at least splitk_min_kb blocks,
    # combined in-launch (0: off)
    # N-sweep kernel (csrc/conv_sweep.hip) for the 1x1 BN-prologue forwards and the folded conv1 data
    # gradients with K <= 256 and OC % 256 == 0, on maps with at least sweep_min_tiles_per_cu 128-row
    # blocks per CU (profiles/r6_sweep/)
    sweep_fwd: bool = True
    sweep_dgrad: bool = False       # (1.08-1.23x per launch, neutral inside the step: off)
    sweep_dgrad_wgs: int = 0        # its persistent grid: 0 one workgroup per CU, N a cap, -1 one per row block
    sweep_min_tiles_per_cu: float = 1.0   # (4: ZeRO-1 -0.6 %; 0.25: TinyImageNet -1.8 %, r6_sweep/ab_threshold.txt)
    splitk_wgs: int = 512
    splitk_min_kb: int = 8           # (4: CIFAR -2.0 %, TinyImageNet -0.3 %; r6_tiny_knobs/confirm.txt)
    tune_table: str = ""            # per-shape tile table (default: ops/tune_table.json)
    tune_modes: str = "all"         # which tune-table sections apply ("none", "fwd,dgrad2", ...)
    # ---- graphs / communication (train/native_step.py, engine/native_trainer.py, parallel/) ----
    graphs: bool = True             # the training step as one HIP graph
    segmented_graphs: bool = False  # per-segment graphs at world 1 (multi-rank rehearsal)
    seg_groups: str = ""            # coarser segmentation of the multi-rank c10d step ("3:3")
    seg_side: bool = True           # batched side stream with late posts in the one-graph multi-rank step
    comm: str = "native"            # native: framework RCCL communicator, one graph; torch: c10d
    comm_side: bool = True          # collectives on the side stream behind their batch (r5_comm_queue/)
    # one-graph multi-rank step where the single-GPU step forks per block: "block" keeps that layout
    # (posts per segment behind its last block batch), "batch" the round-5 batched layout with late posts
    multirank_layout: str = "block"
    comm_loopback: int = 0          # world-1 test aid: all-reduce scales by W, update divides by W
    allreduce_bf16: bool = False    # bf16 gradient all-reduce
    direct_ar: bool = False         # direct two-shot xGMI all-reduce for small buckets (opt-in)
    direct_ar_max_mb: float = 8.0
    rccl_min_ctas: int = 0          # RCCL channel bounds of the framework communicator (0 = RCCL's)
    rccl_max_ctas: int = 0
    # ---- other workloads ----
    frozen_native_head: bool = True  # frozen-backbone trainer: native head kernels
    frozen_graphs: bool = True
    frozen_full_graph: str = "auto"  # auto | 1 | 0: the whole frozen step as one graph
    native_module_graphs: bool = True
    mnist_native: bool = True        # fused HIP MNIST Net
    native_frontends: bool = True    # Accelerate / Composer / Ray facades auto-wrap onto native_module
    policy: StepPolicy = field(default_factory=StepPolicy)

    # ------------------------------------------------------------------------------------------
    def with_(self, **kw) -> "EngineConfig":
        return dataclasses.replace(self, **kw)

    def explicit(self, name: str) -> bool:
        """True when ``name`` was set by the caller (not left to the step-size policy)."""
        return getattr(self, name) is not None

    @classmethod
    def parse(cls, spec: str, base: Optional["EngineConfig"] = None) -> "EngineConfig":
        cfg = dataclasses.replace(base) if base is not None else cls()
        types = {f.name: f.type for f in fields(cls)}
        for item in (spec or "").split(","):
            item = item.strip()
            if not item:
                continue
            if "=" not in item:
                raise ValueError(f"{ENV}: {item!r} is not key=value")
            k, v = (s.strip() for s in item.split("=", 1))
            if k.startswith("policy."):
                pk = k.split(".", 1)[1]
                if pk not in {f.name for f in fields(StepPolicy)}:
                    raise ValueError(f"{ENV}: unknown policy field {pk!r}")
                cfg.policy = dataclasses.replace(cfg.policy, **{pk: float(v)})
                continue
            if k not in types or k == "policy":
                raise ValueError(f"{ENV}: unknown engine field {k!r}")
            setattr(cfg, k, _convert(types[k], v, k))
        return cfg

    @classmethod
    def current(cls) -> "EngineConfig":
        """The process default: dataclass defaults + the ``DBX_ENGINE`` override (re-read when it
        changes, so tests and A/B drivers may set it between builds)."""
        spec = os.environ.get(ENV, "")
        global _CACHE
        if _CACHE is None or _CACHE[0] != spec:
            _CACHE = (spec, cls.parse(spec))
        return _CACHE[1]


_CACHE = None


def _convert(t, v: str, k: str):
    t = str(t)
    if v.lower() in ("none", "auto", "") and "Optional" in t:
        return None
    if "bool" in t:
        if v not in ("0", "1", "true", "false", "True", "False"):
            raise ValueError(f"{ENV}: {k} takes 0 / 1, not {v!r}")
        return v in ("1", "true", "True")
    if "int" in t:
        return int(float(v))
    if "float" in t:
        return float(v)
    return v


def engine_env(**kw) -> str:
    """``DBX_ENGINE`` value for the given fields on top of the current one (A/B drivers, tests)."""
    cur = os.environ.get(ENV, "")
    extra = ",".join(f"{k}={int(v) if isinstance(v, bool) else v}" for k, v in kw.items())
    return ",".join(s for s in (cur, extra) if s)
