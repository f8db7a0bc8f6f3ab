"""Native training step: ResNetProgram + fused optimizer + flat-bucket DDP, replayed as HIP graphs.

One ``NativeTrainer.step()`` = input normalisation (uint8 -> bf16 NHWC4), forward, softmax-CE,
backward, gradient all-reduce (world > 1) and the optimizer update (SGD-momentum / Adam /
AdamW over the flat fp32 master, then the bf16 weight copies are re-derived next step).

Graphs. With world_size == 1 the whole step is ONE captured graph. With world_size > 1 the
step is captured as segments cut where gradient buckets become final (head+layer4 | layer3 |
layer2 | layer1+stem | optimizer); between segment replays the trainer issues the bucket's
RCCL all-reduce on a dedicated comm stream, so the all-reduce of layer4's 15M-parameter bucket
runs under layer3..1's backward (the reference's DDP overlap, SURVEY.md §2.5 M3, without
capturing collectives inside a graph). The optimizer segment waits on the comm stream.

Bucket sizing for xGMI: each segment range is split into chunks of ``bucket_cap_mb`` (default
64 MiB: 8 GPUs x 7 point-to-point links want few, large messages; the 25 MiB NVSwitch-era
default of torch DDP only adds launch latency here).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import Callable, List, Optional, Tuple

import torch
import torch.distributed as dist
import torch.nn as nn

from ..engine_config import EngineConfig
from ..ops import kernels as K
from ..parallel.dist import host_sync_for_gloo
from ..utils import debug as _debug
from ..utils.profiling import PhaseTimer
from .hyper import DeviceHyper
from .program import ResNetProgram, release_dead_graphs


@dataclass
class OptimConfig:
    name: str = "sgd"            # sgd | adam | adamw
    lr: float = 0.1
    momentum: float = 0.9
    dampening: float = 0.0
    nesterov: bool = False
    weight_decay: float = 5e-5
    betas: Tuple[float, float] = (0.9, 0.999)
    eps: float = 1e-8
    grad_clip: float = 0.0       # global-norm clip (DeepSpeed "gradient_clipping")
    trust_coefficient: float = 0.001  # LARS eta (name="lars")


class NativeTrainer:
    def __init__(self, model: nn.Module, batch: int, image_hw: Tuple[int, int], device: torch.device,
                 optim: Optional[OptimConfig] = None, label_smoothing: float = 0.0, use_graphs: bool = True,
                 bucket_cap_mb: float = 64.0, allreduce_dtype: torch.dtype = torch.float32,
                 process_group=None, src_hw: Optional[Tuple[int, int]] = None, mean=None, std=None,
                 zero_stage: int = 0, cutmix_alpha: float = 0.0, seed: int = 0,
                 engine: Optional[EngineConfig] = None):
        self.dev = device
        self.cfg = cfg = engine if engine is not None else EngineConfig.current()
        optim = optim or OptimConfig()
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if (dist.is_available() and dist.is_initialized()) else 1
        if zero_stage and optim.name == "lars":
            raise ValueError("LARS runs on the full flat buffer; use zero_stage=0")
        # ZeRO: segment groups aligned to 16 x world elements (equal per-rank parts) and a flat bf16
        # parameter copy (the all-gather target the weight preparation reads)
        self.prog = ResNetProgram(model, batch, image_hw, device, src_hw=src_hw, mean=mean, std=std,
                                  param_align=16 * self.world if zero_stage else 16, param16=bool(zero_stage),
                                  engine=cfg)
        self.prog.build_backward()
        self.opt = optim
        self.smoothing = label_smoothing
        # CutMix (Composer's CutMix(alpha), `03_composer/01_cifar_composer_resnet.ipynb:430`): per step a
        # batch permutation and one box are sampled here (host, tiny) and applied on the device by the
        # augment kernel (paste) and the CE kernel (mixed soft targets) inside the captured step
        self.cutmix_alpha = float(cutmix_alpha)
        self._rng = __import__("numpy").random.default_rng(seed + 7919 * (dist.get_rank(process_group)
                                                                          if self.world > 1 else 0))
        if self.cutmix_alpha > 0:
            self.prog.enable_cutmix()
        n = self.prog.n_params
        self.mom = torch.zeros(n, device=device)
        self.mom2 = torch.zeros(n, device=device) if optim.name in ("adam", "adamw") else None
        self.hyper = torch.zeros(4, device=device)      # lr, bc1, bc2 (device-side, graph-safe)
        self._hyper_dev = DeviceHyper(self.hyper)
        self.clip_work = torch.zeros(4, device=device)
        self.step_count = 0
        # debug mode synchronizes after every kernel, which graph capture forbids; per-phase
        # profiling (DBX_PROFILE=phases: hipEvent timers + roctx ranges) needs eager phases too
        self.phase_timer = PhaseTimer() if "phases" in os.environ.get("DBX_PROFILE", "").split(",") else None
        self.use_graphs = (use_graphs and device.type == "cuda" and not _debug.enabled()
                           and self.phase_timer is None)
        self.graphs: List[Optional[torch.cuda.CUDAGraph]] = []
        self.bucket_cap = int(bucket_cap_mb * (1 << 20) // 4)
        self.ar_dtype = allreduce_dtype
        # segmented = per-segment graphs + side-stream bucket all-reduces. Always on for world > 1;
        # segmented_graphs forces it at world 1 (with an initialised process group) so the
        # RCCL + capture interplay can be rehearsed on a one-GPU box.
        self.segmented = self.world > 1 or (cfg.segmented_graphs and dist.is_available() and dist.is_initialized())
        self.comm_stream = (torch.cuda.Stream(device=device, priority=-1)
                            if self.segmented and device.type == "cuda" else None)
        # comm "native": the DP bucket all-reduces go through the framework's own RCCL communicator
        # (parallel/comm.py) on the comm stream, and the whole step -- backward segments, forked
        # all-reduces, join, optimizer -- is captured as ONE graph instead of per-segment graphs
        # with eager c10d collectives between replays (ZeRO's reduce-scatter / all-gather included)
        # (RCCL process groups, or a one-rank group: under gloo several ranks share one GPU in the
        # one-box tests, and an RCCL communicator would refuse the duplicate device)
        self.ncomm = None
        if self.segmented and device.type == "cuda" and (self.world == 1 or dist.get_backend(process_group) == "nccl"):
            from ..parallel.comm import native_comm_requested, open_verified_comm
            if native_comm_requested(cfg):
                self.ncomm = open_verified_comm(process_group, device)
        # comm_loopback W (test aid, world 1, DP): the framework communicator's all-reduce scales
        # by W in place -- the sum of W identical replicas -- and the update divides by W, so an
        # ordering bug of the one-graph step (a bucket all-reduced before its gradients are final:
        # invisible at world 1, where the collective is the identity) changes the result
        self.loopback = 1
        self.grad_collectives = "c10d"
        if self.ncomm is not None:
            self.grad_collectives = "framework RCCL communicator"
            from ..parallel.collective_plan import direct_enabled
            # the direct two-shot xGMI path for the ranges the plan prices below the ring (opt-in,
            # direct_ar: unmeasured at world >= 2 until a multi-GPU node runs it)
            lb = cfg.comm_loopback
            if lb > 1 and self.world == 1 and zero_stage == 0:
                self.loopback = self.ncomm.loopback = lb
            if direct_enabled(cfg) and zero_stage == 0 and self.world > 1 and self.ncomm.enable_direct(self.prog.grad):
                self.grad_collectives += " + direct xGMI two-shot (small ranges)"
        # Weight gradients next to the per-segment collectives. In the ONE-graph step (framework
        # communicator) the batched side stream (one fork per backward segment, joined one segment
        # later: overlap_wgrad 2) stays on with LATE posts: segment k's
        # gradient range is final only after segment k+1 joins it, so its all-reduce / reduce-scatter
        # is issued after phase k+1 (the last phase posts the last two ranges). Per-segment graphs
        # (c10d collectives between replays) cannot carry a fork across a graph boundary (a capture
        # must end joined), so there -- and with seg_side off -- the round-3 layout stays: weight
        # gradients in order on the main stream, every range posted right after its own phase
        # (per-gradient forks next to the comm stream cost more than they overlapped:
        # profiles/r2s2_multirank/).
        # The per-block layout (the single-GPU default: one side fork per residual block, lazy joins)
        # keeps its schedule in the one-graph step (multirank_layout "block"): every weight gradient of
        # segment k is queued on the side stream by the end of phase k, so the segment's collective is
        # posted on that same stream right behind its last block batch -- in order, no late post -- and
        # only the ranges whose last gradients run on the main stream in a later phase (layer1's
        # block_tail_main gradients, computed after the stem backward) move to the last phase's post.
        self.block_posts = bool(self.segmented and getattr(self.prog, "side_block_default", False)
                                and cfg.multirank_layout == "block" and self.ncomm is not None
                                and cfg.comm_side and device.type == "cuda")
        if self.segmented and getattr(self.prog, "side_block_default", False) and not self.block_posts:
            # the batched side stream with late posts (round 5's multi-rank layout; the c10d
            # per-segment graphs can carry no fork across a graph boundary)
            p, pol = self.prog, cfg.policy
            p.side_block, p.side_batch = False, True
            p.side_defer = cfg.side_defer if cfg.side_defer is not None else pol.small(p.fwd_flops)
            p.lazy_join = cfg.lazy_join if cfg.lazy_join is not None else pol.tiny(p.fwd_flops)
            p.stem_wg_main = cfg.stem_wg_main if cfg.stem_wg_main is not None else pol.small(p.fwd_flops)
            # (with its collectives on the side stream the batched layout keeps the 64-CU reservation:
            # world-1 RCCL one-graph step with a real collective kernel, headline +0.5-1.1 % over 128,
            # TinyImageNet +0.1 %, profiles/r5_cu_reserve/sweep_late.txt)
            if cfg.side_cu_reserve is None:
                p.side_cu_reserve = 0 if pol.tiny(p.fwd_flops) else 64
        seg_side = cfg.seg_side and (self.ncomm is not None or not self.use_graphs)
        if self.segmented and cfg.overlap_wgrad is None and not seg_side:
            self.prog.overlap_wgrad = False
        self.late_posts = bool(self.segmented and device.type == "cuda" and seg_side and self.prog.overlap_wgrad
                               and self.prog.side_batch)
        if self.segmented and not self.late_posts:
            # per-segment collectives right after their own phase need each segment's weight gradients
            # final at its end: no batched side stream (it joins a segment late)
            self.prog.side_batch = False
        if self.segmented and not cfg.comm_side:
            self.prog.lazy_join = False  # (a separate comm stream orders after the main stream's joins)
        # comm_side (default on): in the one-graph step the collectives run on the weight-gradient
        # side stream itself (behind the batch that finished their range) instead of a third stream.
        # Under DEBUG_HIP_FORCE_GRAPH_QUEUES=2 a separate comm branch took the graph's second hardware
        # queue and pushed the weight-gradient branch onto the main chain's queue: with a real
        # collective in the graph (world-1 comm_loopback=2) TinyImageNet fell from 97.9k to 85.5k
        # img/s and the headline by 1.2 % (profiles/r5_comm_queue/). The joins then wait on an event
        # behind each batch, not on the collectives queued after it.
        self.comm_side = bool(self.ncomm is not None and (self.late_posts or self.block_posts)
                              and device.type == "cuda" and cfg.comm_side)
        if self.comm_side:
            self.comm_stream = self.prog.side_stream()
            self.prog.event_joins = True
            if cfg.side_defer is None:
                self.prog.side_defer = True  # (the side branch then keeps its own hardware queue)
        if self.segmented and ((self.prog.side_block and not self.block_posts) or not self.comm_side):
            # collectives posted per segment need that segment's weight gradients joined at its end
            # (lazy joins only where the collectives ride the side stream behind the batches)
            self.prog.lazy_join = False
        self.flip = None
        self.seg_ranges = self._segment_ranges()
        self.zero = None
        if zero_stage:
            from ..parallel.zero import SegmentedZero
            self.zero = SegmentedZero(self.prog, optim, self.seg_ranges, self.prog.bn_param_blocks(),
                                      stage=zero_stage, process_group=process_group, comm=self.ncomm,
                                      collectives=self.segmented)
            self.mom = self.zero.m  # shard-sized optimizer state only
            self.mom2 = self.zero.v
        self.lars = self._lars_segments() if optim.name == "lars" else None
        self._build_phases()
        self.opt_ranges = self._optimizer_ranges()
        # broadcast initial parameters from rank 0 (DDP constructor semantics, M2)
        if self.world > 1:
            src = 0 if process_group is None else dist.get_global_rank(process_group, 0)
            host_sync_for_gloo(self.prog.master, process_group)
            dist.broadcast(self.prog.master, src, group=process_group)
            for bn in self.prog.bns:
                dist.broadcast(bn.mod.running_mean, src, group=process_group)
                dist.broadcast(bn.mod.running_var, src, group=process_group)
        if self.zero is not None:
            self.zero.refresh_param16()

    # ----------------------------------------------------------------------------------
    def _segment_ranges(self):
        """Contiguous [lo, hi) of every backward segment's gradients (None: no parameters)."""
        out = []
        for rs in self.prog.segment_param_ranges():
            if not rs:
                out.append(None)
                continue
            out.append((min(r[1] for r in rs), max(r[1] + (r[2] + 15) // 16 * 16 for r in rs)))
        return out

    def _build_phases(self):
        """Phases = (name, fn, post): ``fn`` is graph-captured (no collectives); ``post`` is what the
        multi-rank path issues on the comm stream after the phase -- a gradient range (all-reduce,
        or ZeRO reduce-scatter) or a callable (ZeRO norm all-reduce / parameter all-gather)."""
        p = self.prog
        segs = p._segments

        def fwd_phase():
            # bf16 weights + BN-statistics zeroing + every BN's num_batches_tracked, one launch
            p.prepare_weights(step=True)
            p.load_input_u8(self.flip)
            p.forward(smoothing=self.smoothing)

        phases: List[Tuple[str, Callable, Optional[Tuple[int, int]]]] = []
        # phase 0 = forward + first backward segment
        first_name, first_fn = segs[0]
        phases.append(("fwd+" + first_name, lambda: (fwd_phase(), first_fn()), self.seg_ranges[0]))
        for (name, fn), rg in zip(segs[1:], self.seg_ranges[1:]):
            phases.append((name, fn, rg))
        if self.segmented and self.late_posts:
            # batched side stream: phase k completes segment k-1's weight gradients (see __init__)
            rgs = [ph[2] for ph in phases]
            shifted = [None] + rgs[:-1]
            shifted[-1] = [r for r in (rgs[-2], rgs[-1]) if r is not None] if len(rgs) > 1 else rgs[-1]
            phases = [(n, fn, post) for (n, fn, _), post in zip(phases, shifted)]
        elif self.segmented and self.block_posts:
            # per-block layout: each range at its own phase's end, layer1's with the stem's when its last
            # block's tail gradients run on the main stream after the stem backward (see __init__)
            if self.prog.block_tail_main > 0 and len(phases) > 1:
                rgs = [ph[2] for ph in phases]
                shifted = rgs[:-2] + [None, [r for r in (rgs[-2], rgs[-1]) if r is not None]]
                phases = [(n, fn, post) for (n, fn, _), post in zip(phases, shifted)]
        elif self.segmented:
            phases = self._merge_phases(phases)
        z = self.zero
        # ZeRO + clipping with collectives: the shard's sum of squares is all-reduced between phases
        self._zero_norm_separate = z is not None and bool(self.opt.grad_clip) and self.segmented
        if self._zero_norm_separate:
            phases.append(("opt_norm", z.norm_phase, z.allreduce_norm))
        phases.append(("optimizer", self._optimizer_phase, z.gather if z is not None else None))
        self.phases = phases

    def _optimizer_ranges(self):
        """The optimizer inside the backward (engine field ``overlap_optimizer``): SGD / Adam are
        element-wise, so each backward segment's parameters are updated as soon as that segment's
        gradients are final (and, at world > 1, all-reduced), on the weight-gradient side stream right
        behind the segment's last block batch (and its collective) -- the step no longer ends with a
        serial update of every parameter. Per phase the ranges to update after it; the last phase's
        (and layer1's, whose last block's tail weight gradients run on the main stream after the stem
        backward) go on the main stream after the final join; element ranges no segment covers are
        updated in the optimizer phase. Off (None) for clipping / LARS (global norms), ZeRO (its own
        sharded update), the c10d per-segment graphs and the batched side-stream layouts."""
        p, cfg = self.prog, self.cfg
        if not (cfg.overlap_optimizer != 0 and self.zero is None and self.lars is None
                and not (self.opt.grad_clip and self.opt.grad_clip > 0)
                and p.side_block and p.overlap_wgrad and (not self.segmented or self.block_posts)):
            return None
        nph = len(self.seg_ranges)
        per = [[r] if r is not None else [] for r in self.seg_ranges]
        if nph > 1 and p.block_tail_main > 0:
            per[-1] = per[-2] + per[-1]
            per[-2] = []
        if cfg.overlap_optimizer > 0:  # only the first N segments inside the backward
            per = [rs if k < cfg.overlap_optimizer else [] for k, rs in enumerate(per)]
        covered = sorted(r for rs in per for r in rs)
        gaps, pos = [], 0  # (merged: the segments are contiguous in backward order, one launch each gap)
        for lo, hi in covered:
            if lo > pos:
                gaps.append((pos, lo))
            pos = max(pos, hi)
        if pos < p.n_params:
            gaps.append((pos, p.n_params))
        if not covered:
            return None
        return {"per_phase": per, "gaps": gaps}

    def _update_range(self, lo: int, hi: int):
        p, o = self.prog, self.opt
        gscale = 1.0 / (self.world * self.loopback)
        if o.name == "sgd":
            K.sgd_step(p.master[lo:hi], p.grad[lo:hi], self.mom[lo:hi], None, lr=o.lr, momentum=o.momentum,
                       dampening=o.dampening, weight_decay=o.weight_decay, nesterov=o.nesterov, first=False,
                       grad_scale=gscale, hyper=self.hyper)
        else:
            K.adam_step(p.master[lo:hi], p.grad[lo:hi], self.mom[lo:hi], self.mom2[lo:hi], None, lr=o.lr,
                        beta1=o.betas[0], beta2=o.betas[1], eps=o.eps, weight_decay=o.weight_decay,
                        decoupled=(o.name == "adamw"), step=1, grad_scale=gscale, hyper=self.hyper)

    def _after_phase_updates(self, i: int):
        """Issue phase i's parameter updates (see _optimizer_ranges)."""
        if self.opt_ranges is None:
            return
        rs = self.opt_ranges["per_phase"][i] if i < len(self.opt_ranges["per_phase"]) else []
        if not rs:
            return
        last = i == len(self.opt_ranges["per_phase"]) - 1
        if self.dev.type != "cuda" or last:
            for r in rs:  # (the last phase ended with the final join: on the main stream)
                self._update_range(*r)
            return
        run = (lambda rs=rs: [self._update_range(*r) for r in rs])
        if not self.prog.defer_on_side(run):  # behind the deferred batch (and collective), or now
            side = self.prog.side_stream()
            side.wait_stream(torch.cuda.current_stream(self.dev))
            with torch.cuda.stream(side):
                run()
            self.prog._side_pending = True  # (the next join, at the latest the final one, waits for it)

    def _merge_phases(self, phases):
        """Optional coarser graph segmentation of the multi-rank path: seg_groups "3:3" merges
        the six backward segments into two graphs (one all-reduce cut after layer3). Default: one
        graph per backward segment. Measured over RCCL on one MI355X (world-1 process group with
        segmented_graphs=1, ResNet-50 b1024, wgrad side stream on): 6 segments 13.98k / 14.03k
        img/s, 2 segments 14.05k / 14.07k, one backward graph 13.99k / 14.00k, plain single graph
        14.45k / 14.43k (profiles/r2s2_multirank/step_layout_ab.txt) -- boundaries are not what
        the segmented path cost: the wgrad side stream next to the comm streams was (now off in
        this mode, see __init__). The finer split (more overlap, smallest exposed tail) stays.
        Groups merge only when their gradient ranges are disjoint and in order."""
        spec = self.cfg.seg_groups
        if not spec:
            return phases
        sizes = [int(x) for x in spec.split(":") if x.strip()]
        sizes = [x for x in sizes if x > 0]
        if sum(sizes) != len(phases):
            raise ValueError(f"seg_groups={spec!r} does not cover {len(phases)} backward segments")
        merged, pos = [], 0
        for sz in sizes:
            grp = phases[pos:pos + sz]
            pos += sz
            rgs = sorted(rg for _, _, rg in grp if rg is not None)
            # consecutive phases own consecutive parameter groups (at most alignment padding between)
            if any(a[1] > b[0] for a, b in zip(rgs, rgs[1:])):
                return phases  # non-adjacent gradient ranges: keep one segment per phase
            fns = [fn for _, fn, _ in grp]
            merged.append(("+".join(nm for nm, _, _ in grp),
                           (lambda fns=fns: [f() for f in fns]),
                           (rgs[0][0], rgs[-1][1]) if rgs else None))
        return merged

    def _lars_segments(self):
        """Per-tensor segments of the flat buffer for LARS; conv / fc weights are adapted (and decayed),
        BN affine parameters and biases are not (the usual large-batch recipe)."""
        rs = self.prog.param_ranges
        dev = self.dev
        off = torch.tensor([r[1] for r in rs], dtype=torch.int32, device=dev)
        ln = torch.tensor([r[2] for r in rs], dtype=torch.int32, device=dev)
        bn_names = {f"{bn.name}." for bn in self.prog.bns}
        adapt = torch.tensor([int(r[0].endswith(".weight") and not any(r[0].startswith(b) for b in bn_names))
                              for r in rs], dtype=torch.int32, device=dev)
        return off, ln, adapt, torch.zeros(K.LARS_MAX_BLOCKS * 2 * len(rs), device=dev, dtype=torch.float64), max(r[2] for r in rs)

    def _optimizer_phase(self):
        p, o = self.prog, self.opt
        if self.zero is not None:
            # ZeRO-1/2: update this rank's shard of the fp32 master with its shard of the optimizer
            # state (the reduce-scatter and the all-gather run around this phase, not inside it:
            # the phase is captured at every world size). lr / bias corrections come from the
            # device-side hyper tensor so a replayed step follows set_lr() and the step count.
            if o.grad_clip and not self._zero_norm_separate:
                self.zero.norm_phase()
            self.zero.update(hyper=self.hyper)
            return
        if self.opt_ranges is not None:  # updated inside the backward: only uncovered ranges remain
            for r in self.opt_ranges["gaps"]:
                self._update_range(*r)
            return
        gsp = None
        gdiv = self.world * self.loopback  # the reduced gradient is a sum over gdiv replicas
        if o.grad_clip and o.grad_clip > 0:
            # clip on the averaged gradient: factor computed on device (no host sync)
            K.global_norm_clip_factor(p.grad, o.grad_clip * gdiv, self.clip_work)
            gsp = self.clip_work[2:3]
        if self.lars is not None:
            # the clip factor scales the gradient before the trust ratios, as torch's
            # clip_grad_norm_ + LARS does on the autograd engine
            if gsp is not None:
                p.grad.mul_(gsp)
            off, ln, adapt, norms, mx = self.lars
            K.lars_scale(p.master, p.grad, off, ln, adapt, norms, grad_scale=1.0 / gdiv,
                         eta=o.trust_coefficient, weight_decay=o.weight_decay, max_len=mx)
            K.sgd_step(p.master, p.grad, self.mom, None, lr=o.lr, momentum=o.momentum, dampening=o.dampening,
                       weight_decay=0.0, nesterov=o.nesterov, first=False, grad_scale=1.0, hyper=self.hyper)
            return
        gscale = 1.0 / gdiv
        if o.name == "sgd":
            K.sgd_step(p.master, p.grad, self.mom, None, lr=o.lr, momentum=o.momentum, dampening=o.dampening,
                       weight_decay=o.weight_decay, nesterov=o.nesterov, first=False, grad_scale_ptr=gsp,
                       grad_scale=gscale, hyper=self.hyper)
        else:
            K.adam_step(p.master, p.grad, self.mom, self.mom2, None, lr=o.lr, beta1=o.betas[0], beta2=o.betas[1],
                        eps=o.eps, weight_decay=o.weight_decay, decoupled=(o.name == "adamw"), step=1,
                        grad_scale_ptr=gsp, grad_scale=gscale, hyper=self.hyper)

    # ----------------------------------------------------------------------------------
    def _post(self, post):
        if post is None:
            return
        if callable(post):
            post()
        elif isinstance(post, list):  # late posts: several gradient ranges after one phase
            for rg in post:
                self._post(rg)
        elif self.zero is not None:
            self.zero.reduce_range(*post)
        else:
            self._allreduce_range(*post)

    def _allreduce_range(self, lo: int, hi: int):
        g = self.prog.grad
        if self.ncomm is not None:  # enqueued on the current (comm) stream; capturable
            from ..parallel.collective_plan import plan_allreduce
            esz = torch.tensor([], dtype=self.ar_dtype).element_size()
            plan = plan_allreduce(hi - lo, esz, self.world, self.bucket_cap,
                                  allow_direct=self.ncomm.direct is not None and self.ar_dtype == torch.float32)
            for a, b in plan.buckets:
                chunk = g[lo + a:lo + b]
                if self.ar_dtype == torch.float32:
                    self.ncomm.all_reduce(chunk)  # direct path when the plan picked it (NativeComm.all_reduce)
                else:
                    buf = chunk.to(self.ar_dtype)
                    self.ncomm.all_reduce(buf)
                    chunk.copy_(buf)
            return
        host_sync_for_gloo(g, self.pg)
        pos = lo
        while pos < hi:
            end = min(hi, pos + self.bucket_cap)
            chunk = g[pos:end]
            if self.ar_dtype == torch.float32:
                dist.all_reduce(chunk, group=self.pg)
            else:
                buf = chunk.to(self.ar_dtype)
                dist.all_reduce(buf, group=self.pg)
                chunk.copy_(buf)
            pos = end

    def _sample_cutmix(self):
        """lam ~ Beta(a, a); box of area (1 - lam) at a uniform centre, clipped; lam re-derived from
        the clipped area (Composer's CutMix); one permutation of the batch."""
        p, r = self.prog, self._rng
        H, W = p.H, p.W
        lam = float(r.beta(self.cutmix_alpha, self.cutmix_alpha))
        cut = (1.0 - lam) ** 0.5
        ch, cw = int(H * cut), int(W * cut)
        cy, cx = int(r.integers(0, H)), int(r.integers(0, W))
        y0, y1 = min(max(cy - ch // 2, 0), H), min(max(cy + ch // 2, 0), H)
        x0, x1 = min(max(cx - cw // 2, 0), W), min(max(cx + cw // 2, 0), W)
        lam = 1.0 - (y1 - y0) * (x1 - x0) / float(H * W)
        perm = torch.from_numpy(r.permutation(p.N).astype("int32"))
        box = torch.tensor([y0, y1, x0, x1], dtype=torch.int32)
        lamt = torch.tensor([lam], dtype=torch.float32)
        if self.dev.type == "cuda":
            perm, box, lamt = perm.pin_memory(), box.pin_memory(), lamt.pin_memory()
        self._mix_host = (perm, box, lamt)  # keep the pinned sources alive until the copies ran
        p.mix_perm.copy_(perm, non_blocking=True)
        p.mix_box.copy_(box, non_blocking=True)
        p.mix_lam.copy_(lamt, non_blocking=True)

    def _set_hyper(self):
        o = self.opt
        self.step_count += 1
        t = self.step_count
        if o.name in ("sgd", "lars"):
            vals = [o.lr, 1.0, 1.0, 0.0]
        else:
            vals = [o.lr, 1.0 - o.betas[0] ** t, 1.0 - o.betas[1] ** t, 0.0]
        self._hyper_dev.set(vals)

    def set_lr(self, lr: float):
        self.opt.lr = float(lr)

    def _waits_comm(self, i: int, name: str) -> bool:
        # the optimizer phases consume the reduced gradients / norm; the first phase of a step
        # consumes the previous step's all-gathered parameters
        # (inside the one-graph capture the comm stream joins only after its first fork: no wait on
        # work recorded outside the capture)
        first = i == 0 and not getattr(self, "_capturing_one", False)
        return self.segmented and (first or name in ("optimizer", "opt_norm"))

    def _run_phases_eager(self):
        if self.dev.type != "cuda":  # CPU (reference ops; gloo collectives, synchronous)
            for i, (name, fn, post) in enumerate(self.phases):
                fn()
                if self.segmented:
                    self._post(post)
                self._after_phase_updates(i)
            return
        cur = torch.cuda.current_stream(self.dev)
        for i, (name, fn, post) in enumerate(self.phases):
            if self._waits_comm(i, name):
                self.prog.launch_pending()
                cur.wait_stream(self.comm_stream)
            if self.phase_timer is not None:
                with self.phase_timer.phase(name):
                    fn()
            else:
                fn()
            if post is not None and self.segmented:
                # (comm_side with a deferred side batch: the collective goes in behind the batch,
                # under the batch's fork event -- the main stream's state at this phase's end)
                if not (self.comm_side and self.prog.defer_on_side(lambda post=post: self._post(post))):
                    self.comm_stream.wait_stream(cur)
                    with torch.cuda.stream(self.comm_stream):
                        self._post(post)
            self._after_phase_updates(i)

    def _graph_phases(self):
        return self.phases

    def _capture(self):
        """Capture each phase (or the whole step when not segmented) into HIP graphs."""
        release_dead_graphs(self.dev)
        s = torch.cuda.Stream(device=self.dev)
        s.wait_stream(torch.cuda.current_stream(self.dev))
        pool = torch.cuda.graph_pool_handle()
        self.graphs = []
        # thread-local capture whenever a process group exists: its watchdog thread polls the
        # completion events of earlier collectives while we capture, and under the default
        # global mode such a query from another thread invalidates the capture
        mode = "thread_local" if (dist.is_available() and dist.is_initialized()) else "global"
        with torch.cuda.stream(s):
            if self.ncomm is not None:
                # one graph: the comm-stream fork / join of every bucket is recorded as graph edges
                g = torch.cuda.CUDAGraph()
                self._capturing_one = True
                try:
                    with torch.cuda.graph(g, pool=pool, stream=s, capture_error_mode=mode):
                        self._run_phases_eager()
                        self.prog.launch_pending()
                        torch.cuda.current_stream(self.dev).wait_stream(self.comm_stream)
                finally:
                    self._capturing_one = False
                self.graphs = [g]
            elif not self.segmented:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=pool, stream=s, capture_error_mode=mode):
                    for i, (_, fn, _) in enumerate(self.phases):
                        fn()
                        self._after_phase_updates(i)
                    self.prog.launch_pending()
                self.graphs = [g]
            else:
                for _, fn, _ in self._graph_phases():
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, pool=pool, stream=s, capture_error_mode=mode):
                        fn()
                    self.graphs.append(g)
        torch.cuda.current_stream(self.dev).wait_stream(s)
        torch.cuda.synchronize(self.dev)

    def _replay(self):
        cur = torch.cuda.current_stream(self.dev)
        if not self.segmented or self.ncomm is not None:
            if self.ncomm is not None:
                cur.wait_stream(self.comm_stream)  # eager warm-up collectives
            self.graphs[0].replay()
            return
        for i, ((name, _, post), g) in enumerate(zip(self._graph_phases(), self.graphs)):
            if self._waits_comm(i, name):
                cur.wait_stream(self.comm_stream)
            g.replay()
            if post is not None:
                self.comm_stream.wait_stream(cur)
                with torch.cuda.stream(self.comm_stream):
                    self._post(post)

    # ----------------------------------------------------------------------------------
    def step(self, images_u8: Optional[torch.Tensor] = None, labels: Optional[torch.Tensor] = None,
             boxes: Optional[torch.Tensor] = None, flips: Optional[torch.Tensor] = None):
        """One training step. ``images_u8`` [N,Hs,Ws,C] uint8, ``labels`` [N] int64, optional
        crop ``boxes`` [N,4] / ``flips`` [N] are copied into the program's static input buffers
        (pass None to reuse what is already there)."""
        p = self.prog
        p.training = True
        if images_u8 is not None:
            p.img_u8.copy_(images_u8, non_blocking=True)
        if labels is not None:
            p.labels.copy_(labels, non_blocking=True)
        if boxes is not None:
            p.boxes.copy_(boxes, non_blocking=True)
        if flips is not None:
            p.flip.copy_(flips, non_blocking=True)
        if self.cutmix_alpha > 0:
            self._sample_cutmix()
        self._set_hyper()
        try:
            self._step_inner()
        except BaseException:
            p.drop_pending()  # a side batch deferred by the failed step must not launch later
            raise
        if self.zero is not None:
            # a replayed graph does not run zero.step() in Python: keep its counter (saved in
            # ZeRO checkpoints) on the trainer's
            self.zero.step_count = self.step_count

    def _step_inner(self):
        if not self.use_graphs:
            self._run_phases_eager()
            return
        if not self.graphs:
            # two eager warm-up steps (allocator / library handles), then capture. The warm-up
            # steps are real steps: they update weights like any other.
            if not hasattr(self, "_warm"):
                self._warm = 0
            if self._warm < 2:
                self._warm += 1
                self._run_phases_eager()
                return
            # stream capture records without executing: no state to snapshot
            self._capture()
        self._replay()

    # ----------------------------------------------------------------------------------
    @torch.no_grad()
    def evaluate_batch(self, images_u8: torch.Tensor, labels: torch.Tensor,
                       boxes: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Eval-mode forward (running BN stats); returns logits (bf16) and accumulates metrics.
        A short final batch is padded (padding rows get label -> excluded by the caller)."""
        p = self.prog
        p.training = False
        if self.comm_stream is not None:  # the last step's parameter all-gather (ZeRO)
            torch.cuda.current_stream(self.dev).wait_stream(self.comm_stream)
        n = images_u8.shape[0]
        p.img_u8[:n].copy_(images_u8)
        p.labels[:n].copy_(labels)
        if boxes is not None:
            p.boxes[:n].copy_(boxes)
        p.flip.zero_()
        p.prepare_weights()
        p.load_input_u8(None)
        out = p.forward(smoothing=0.0, compute_grad=False, metrics=False)
        p.training = True
        return out[:n]

    def sync_master(self) -> None:
        """Make the module's fp32 parameters (views of the flat master) complete on every rank:
        under ZeRO each rank only updates its shard (collective; call on all ranks before a
        checkpoint / state_dict)."""
        if self.zero is not None:
            if self.dev.type == "cuda" and self.comm_stream is not None:
                torch.cuda.current_stream(self.dev).wait_stream(self.comm_stream)
            self.zero.gather_master()

    def params_changed(self) -> None:
        """Call after writing the parameters from outside (checkpoint load): ZeRO re-derives its
        bf16 parameter copy from the (full) fp32 master."""
        if self.zero is not None:
            self.zero.refresh_param16()

    def read_metrics(self, reset: bool = True) -> Tuple[float, float]:
        m = self.prog.metrics[:2].tolist()
        if reset:
            self.prog.metrics.zero_()
        return m[0], m[1]
