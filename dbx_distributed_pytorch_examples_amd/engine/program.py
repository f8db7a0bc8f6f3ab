"""ResNet programs: a static NHWC-bf16 forward/backward schedule over the HIP kernels.

The reference trains torchvision ResNets through autograd + cuDNN (SURVEY.md §3.3 hot loop).
On MI355X we instead *compile* the module tree once into a fixed op list over a preallocated
activation arena, because that is what lets the hot path be fused and graph-captured:

* the BN of every conv is split into (stats in the conv epilogue) + (apply in the consumer's
  prologue), so no BN/ReLU output is ever materialised inside a block; the block tail
  (BN + residual [+ BN of the downsample branch] + ReLU) is one pass;
* backward is written out explicitly: BN-backward reductions with recomputed ReLU masks,
  dgrad with the residual gradient accumulated in its epilogue, split-K wgrad whose reduce
  writes fp32 straight into the flat gradient buffer (= the DDP buckets);
* every tensor has a fixed address, so the whole step (weight cast -> fwd -> loss -> bwd ->
  optimizer) replays as a HIP graph (``engine.step``), segmented at the points where gradient
  buckets become ready so RCCL all-reduces overlap the remaining backward.

Parameters live in ONE flat fp32 master buffer (conv weights in KRSC order); the module's
``nn.Parameter`` s are re-pointed at views of it (``.data`` swap: the Parameter objects, and any
optimizer already holding them, stay valid; conv weights as channels_last views), so
``model.state_dict()`` / ``load_state_dict`` / checkpoint files keep torchvision layouts.

Supported module trees: ``models.ResNet`` (BasicBlock / Bottleneck, any in_channels <= 4) and
``models.CifarResNet18``; everything else trains through the autograd path (engine.autograd_step).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn

from ..engine_config import EngineConfig
from ..models.resnet import BasicBlock, Bottleneck, CifarBlock, CifarResNet18, ResNet
from ..ops import kernels as K

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def _repoint(p: nn.Parameter, view: torch.Tensor) -> None:
    """Make the EXISTING Parameter object a view of the flat master (``.data`` swap): optimizers and
    hooks created on the module before compilation keep working on the live weights."""
    p.data = view
    if p.grad is not None and (p.grad.device != view.device or p.grad.shape != view.shape):
        p.grad = None
    elif p.grad is not None and p.grad.stride() != view.stride():
        # a gradient accumulated before compilation (e.g. a first batch on the torch module) keeps
        # its values in the parameter's NEW layout (KRSC: channels-last), or every later accumulation
        # into it breaks autograd's gradient layout contract
        g = torch.empty_strided(view.shape, view.stride(), dtype=p.grad.dtype, device=view.device)
        g.copy_(p.grad)
        p.grad = g


def supports(model: nn.Module) -> bool:
    if not isinstance(model, (ResNet, CifarResNet18)):
        return False
    if model.conv1.in_channels > 4:
        return False
    return True


def release_dead_graphs(dev) -> None:
    """Before a capture: destroy the captured graphs of dead trainers / programs (reference cycles
    keep them until a GC pass) and drain the device after it. Graph teardown left to the collector
    inside torch.cuda.graph's own enter (no device sync after it), or to a GC pass while another
    thread replays, was followed by host crashes in the next graph launch on the GPU box
    (profiles/r4_final2/README.md)."""
    import gc

    from .. import check_graph_queues
    check_graph_queues()
    gc.collect()
    torch.cuda.synchronize(dev)


# ======================================================================================
# specs
# ======================================================================================

@dataclass
class ConvL:
    name: str
    mod: nn.Conv2d
    IC: int
    OC: int
    R: int
    S: int
    stride: int
    pad: int
    IH: int
    IW: int
    OH: int
    OW: int
    stem: bool = False
    off: int = 0          # master offset (KRSC fp32)
    w16: Optional[torch.Tensor] = None   # [OC, KTOT] bf16 forward weights
    wt16: Optional[torch.Tensor] = None  # [IC, R*S*OC] bf16 dgrad weights
    grad: Optional[torch.Tensor] = None  # fp32 [OC, R*S*IC] view into the flat grad buffer

    @property
    def numel(self) -> int:
        return self.OC * self.IC * self.R * self.S


@dataclass
class BNL:
    name: str
    mod: nn.BatchNorm2d
    C: int
    off_w: int = 0
    off_b: int = 0
    # per-step device state (views into one fp32 arena)
    scale: Optional[torch.Tensor] = None
    shift: Optional[torch.Tensor] = None
    mean: Optional[torch.Tensor] = None
    invstd: Optional[torch.Tensor] = None
    coeff: Optional[torch.Tensor] = None
    stats: Optional[torch.Tensor] = None
    bstats: Optional[torch.Tensor] = None
    gamma: Optional[torch.Tensor] = None
    beta: Optional[torch.Tensor] = None
    dgamma: Optional[torch.Tensor] = None
    dbeta: Optional[torch.Tensor] = None


@dataclass
class BlockL:
    kind: str                      # "bottleneck" | "basic"
    convs: List[ConvL]
    bns: List[BNL]
    ds_conv: Optional[ConvL]
    ds_bn: Optional[BNL]
    in_shape: Tuple[int, int, int]   # H, W, C of the block input
    out_shape: Tuple[int, int, int]
    # activations
    ys: List[torch.Tensor] = field(default_factory=list)   # raw conv outputs
    # relu(bn(ys[j])) for j < nconv-1 when conv j+1 can write it back (stride 1): its wgrad input
    acts: List[Optional[torch.Tensor]] = field(default_factory=list)
    yd: Optional[torch.Tensor] = None
    out: Optional[torch.Tensor] = None
    # gradients
    dys: List[torch.Tensor] = field(default_factory=list)  # BN-input grads (per conv)
    das: List[torch.Tensor] = field(default_factory=list)  # grads wrt intermediate activations
    dyd: Optional[torch.Tensor] = None
    dsbuf: Optional[torch.Tensor] = None
    dx: Optional[torch.Tensor] = None                       # grad wrt block input


class ResNetProgram:
    """Compile a ResNet nn.Module into a fixed-shape NHWC program for (batch, H, W)."""

    def __init__(self, model: nn.Module, batch: int, image_hw: Tuple[int, int], device: torch.device,
                 src_hw: Optional[Tuple[int, int]] = None, mean=None, std=None, param_align: int = 16,
                 param16: bool = False, engine: Optional[EngineConfig] = None):
        """``image_hw``: network input size; ``src_hw``: size of the uint8 images handed in
        (crop/resize to image_hw happens on the GPU, ``augment_u8``); default = image_hw.
        ``param_align``: every backward segment's parameter group starts on a multiple of this many
        elements (ZeRO: 16 x world, so a segment splits into equal per-rank parts); ``param16``:
        keep a flat bf16 copy of the parameters (``self.param16``, ZeRO's all-gather target) and
        derive the compute weights from it instead of from the fp32 master. ``engine``: the schedule /
        fusion switches (default ``EngineConfig.current()``; its ``None`` fields are resolved here by
        the step-size policy)."""
        if not supports(model):
            raise TypeError(f"ResNetProgram does not support {type(model).__name__}")
        self.model = model
        self.N = batch
        self.H, self.W = image_hw
        self.src_hw = tuple(src_hw) if src_hw else (self.H, self.W)
        self.norm_mean = tuple(mean) if mean else None
        self.norm_std = tuple(std) if std else None
        self.dev = device
        self.in_ch = model.conv1.in_channels
        self.cfg = cfg = engine if engine is not None else EngineConfig.current()
        pol = cfg.policy
        ow = cfg.overlap_wgrad
        # weight gradients on a side stream (overlap_wgrad None / 2: batched, one fork per backward
        # segment -- see self.side_batch; "1": one fork per weight gradient; "0": in order on the main
        # stream). Per-gradient forks cost more than they overlap on launch-bound steps (ResNet-18 CIFAR
        # b256 189k img/s vs 222k in order) while one fork per segment wins at every size: CIFAR
        # 229-230k, TinyImageNet 95.3-95.5k vs 90.6-91.5k, headline 16.07-16.15k vs 15.94-15.99k
        # (profiles/r3s2_batched/)
        self.overlap_wgrad = ow != 0
        # (the in-launch split-K reduce and the producer-side BN finalize (K.BnFin) measured slower than
        # the launches they remove on all three presets and were removed in round 6: profiles/r3s2_fuse_ab/;
        # the finalize re-measured after the round-6 changes: -4 % to -8 %, profiles/r6_fuse_fin/)
        self.fuse_fin = False

        # store block-internal BN outputs from the MASK_Y dgrad epilogue for the wgrads
        self.act_writeback = cfg.act_writeback
        # compute block outputs inside the next block's conv1 prologue instead of a bn_apply pass
        self.fuse_tail = cfg.fuse_tail
        self.pool_reduce = cfg.pool_reduce
        # BN-backward apply of a 1x1 conv's output BN computed in that conv's dgrad prologue
        self.fuse_bwd_apply = cfg.fuse_bwd_apply
        # ... only for large operands: folding orders the wgrad after the dgrad (no overlap), which
        # costs more than the saved pass when the kernels are too small to fill the GPU
        self.fold_min = cfg.fold_min_elems if cfg.fold_min_elems is not None else 1 << 25
        # ... and only where the dgrad's output channels (N) are at most this multiple of its
        # reduction channels: every N tile of a folded dgrad re-reads and re-applies the operand
        # (default 1: the bottleneck conv1 dgrads, N = 4K, stay unfolded -- 14.39-14.41k vs
        # 14.22-14.27k img/s folded, ResNet-50 b1024, profiles/r2s3_fold/fold_ratio_ab.txt)
        self.fold_max_ratio = cfg.fold_max_ratio if cfg.fold_max_ratio is not None else 1.0
        # ... except at feature maps >= this size (the ratio limit is about the N-tile repeats of
        # the operand prologue: at 56x56 the conv1 dgrads have only 1-2 N tiles; 15.19k / 15.21k vs
        # 15.17k / 15.13k img/s with the limit everywhere, profiles/r2s3_fold/fold_ratio_ab.txt)
        self.fold_ratio_min_hw = cfg.fold_ratio_min_hw
        # bottleneck conv3 backward as ONE kernel (BN3-backward apply + dgrad + MASK_Y epilogue +
        # weight gradient, K.conv_dwfused): dy3 and the BN2 output a2 never reach HBM
        self.fuse_dw = cfg.fuse_dw
        # stem backward as ONE kernel (max-pool backward + BN-backward apply + stem weight gradient,
        # K.stem_bwd_fused): the full-resolution stem gradient never reaches HBM. Off by default: it
        # saves the 3.3 GB dy0 round trip at b1024 but runs 1.97 ms against 0.91 + 0.92 ms for the
        # streaming pool/BN pass + the stem wgrad (the 4-window argmax routing per element is VALU work
        # that the two-workgroups-per-CU MFMA kernel cannot hide; profiles/r2s4_stem/)
        self.fuse_stem_bwd = cfg.fuse_stem_bwd
        # 3x3 convs whose plain-operand shape has an eight-wave kernel entry (ops/tune_table.json "fwd0",
        # csrc/conv_fast.hip): the forward materialises the input BN output relu(bn(y)) once (the
        # block's acts buffer, which backward needs anyway) and runs the conv without a prologue
        # (the same for the bottleneck's 1x1 conv3 measured -0.3 %: profiles/r3s2_hipenv/fast_mat1_ab.txt)
        self.fast_mat = cfg.fast_mat
        self._wstream = None
        self._side_pending = False
        # overlap_wgrad 2: the side stream forks once per backward segment (batched) instead
        # of once per weight gradient. Callers that need every segment's gradients final at its end
        # (per-segment all-reduces: NativeTrainer / native_module at world > 1) turn it off.
        self.side_batch = ow in (None, 2) and not self.fuse_stem_bwd  # (shares self.ws)
        # 3: one fork per residual block (after its data gradients), every segment joined at its end:
        # overlap that keeps segment-final gradients (the per-segment all-reduces at world > 1)
        self.side_block = ow == 3 and not self.fuse_stem_bwd
        self._side_q = []
        self.param_align = max(16, int(param_align))
        self._want_param16 = param16
        self._build_layers()
        # consumer-side forward BN finalize (K.conv_fwd fin_in): each workgroup of the
        # consuming conv re-reads the statistics shards (2 x NSHARD x C doubles). Off: measured slower
        # than the finalize launch it removes even on the launch-bound CIFAR step (212-214k vs 222k
        # img/s; TinyImageNet 87.6k vs 89.5-89.9k, profiles/r3s2_finin/)
        fl = self.fwd_conv_flops()
        self.fwd_flops = fl
        self.fin_in = bool(cfg.fin_in)
        # Launch-bound small steps (< 0.5 TFLOP of forward conv work: the CIFAR / TinyImageNet presets)
        # keep 4 statistics shards per BN instead of NSHARD, which makes the consumer-side forward
        # finalize cheap enough to replace the bn_finalize launches: CIFAR 233.7-236.6k vs 229.1-231.0k,
        # TinyImageNet 96.9-97.1k vs 95.4-96.0k img/s; the b1024 headline keeps NSHARD and standalone
        # finalizes (16.14k with them vs 16.38-16.40k; profiles/r4_s6/, r4_s7/). nshard / fin_in set
        # explicitly win.
        self.small_step = pol.small(fl)
        self.nshard = cfg.nshard if cfg.nshard is not None else (4 if self.small_step else K.NSHARD)
        # (round 6: only the launch-bound CIFAR class keeps it; the TinyImageNet class runs the finalize
        # launches again after the round-5/6 schedule changes: 105,548 / 105,605 vs 105,038 / 104,844
        # img/s, profiles/r6_tiny_fin/)
        if pol.tiny(fl) and cfg.fin_in is None:
            self.fin_in = True
        # consumer-side backward finalize: a BN-backward apply pass computes its coefficients from the
        # moment shards itself (K.bn_bwd_apply fin=) instead of a bn_bwd_coeff launch in front of it
        # (on by default for the small steps with 4-shard slabs: CIFAR 238.2-238.6k vs 233.7k img/s
        # without it; at NSHARD = 32 every block of an apply would re-read 64 doubles per channel:
        # profiles/r4_s7/); at 50-500 GFLOP (TinyImageNet) only for BNs of <= 512 channels: 95.7-95.9k vs 95.5k img/s
        # (all widths 94.7k: an apply that finalizes in-launch is capped near C x 512 channel-finalizes,
        # few blocks at 2048); CIFAR keeps every width (253.1-254.0k vs 251.6-252.5k at <= 256):
        # profiles/r4_s18/. coeff_in_maxc overrides the width limit (0: none).
        # by default the side stream forks once per residual BLOCK (overlap_wgrad 3; first from 50
        # GFLOP of forward conv work up, TinyImageNet and ImageNet) -- with the deferred launch and lazy joins below
        # that fills the windows where the batched side stream waited for its next fork: headline
        # 16,755-16,865 vs 16,709-16,731, TinyImageNet 100.4-100.8k vs 99.4k img/s (CIFAR neutral at
        # first): profiles/r5_side_defer/mode3.txt. The multi-rank trainer puts the batched layout back
        # (its collectives are posted per segment).
        # (late in round 5, with the block tails on the main stream and the downsample forward on the side
        # stream, the CIFAR class gains too: 267.4-267.8k vs 262.3-263.0k img/s, profiles/r5_side_defer/
        # cifar_late.txt -- the per-block default now covers every step size)
        self.side_block_default = ow is None and not self.fuse_stem_bwd and self.overlap_wgrad
        if self.side_block_default:
            self.side_block, self.side_batch = True, False
        self.coeff_in = cfg.coeff_in if cfg.coeff_in is not None else (pol.small(fl) and self.nshard <= 4)
        mc = cfg.coeff_in_maxc
        self.coeff_in_maxc = (mc or None) if mc is not None else (None if pol.tiny(fl) else 512)
        # split-K weight-gradient reductions of a side-stream batch deferred to two launches at its end
        # (K.ReduceBatch; 19 reduce launches per CIFAR step): on for the smallest steps (< 50 GFLOP),
        # CIFAR 252.7-253.8k vs 243.7-245.5k img/s; TinyImageNet loses (93.3-93.8k vs 95.4k: its
        # larger slabs leave L2 before the batch-end reduce), profiles/r4_s12/
        self.defer_reduce = cfg.defer_reduce if cfg.defer_reduce is not None else pol.tiny(fl)
        self.wred_arena = torch.empty(0, device=device, dtype=torch.float32)
        self._wred_off = 0
        if not self.overlap_wgrad:
            # without the side stream folding costs no overlap: fold every BN-backward apply it can
            # (unless set explicitly) -- CIFAR b256 193.7k vs 189.5k img/s with overlap (r3s2_knobs)
            if cfg.fold_min_elems is None:
                self.fold_min = 0
            if cfg.fold_max_ratio is None:
                self.fold_max_ratio = 8.0
        self._alloc_params()
        self._alloc_activations()
        self.build_fins()
        self._pack_step_descs()
        self.training = True

    # ----------------------------------------------------------------------------------
    # construction
    # ----------------------------------------------------------------------------------
    def _conv(self, name, mod: nn.Conv2d, ih, iw, stem=False) -> ConvL:
        R, S = mod.kernel_size
        st, pad = mod.stride[0], mod.padding[0]
        if mod.bias is not None or mod.groups != 1 or mod.dilation != (1, 1) or mod.stride[0] != mod.stride[1]:
            raise TypeError(f"{name}: unsupported conv configuration")
        oh, ow = K.conv_out_hw(ih, iw, R, S, st, pad)
        return ConvL(name, mod, mod.in_channels, mod.out_channels, R, S, st, pad, ih, iw, oh, ow, stem)

    def _build_layers(self):
        m = self.model
        self.stem = self._conv("conv1", m.conv1, self.H, self.W, stem=True)
        self.stem_bn = BNL("bn1", m.bn1, m.bn1.num_features)
        mp = m.maxpool
        self.pool_k, self.pool_s, self.pool_p = mp.kernel_size, mp.stride, mp.padding
        ph = (self.stem.OH + 2 * self.pool_p - self.pool_k) // self.pool_s + 1
        pw = (self.stem.OW + 2 * self.pool_p - self.pool_k) // self.pool_s + 1
        self.pool_hw = (ph, pw)
        h, w, c = ph, pw, self.stem.OC
        self.blocks: List[BlockL] = []
        for li in range(1, 5):
            layer = getattr(m, f"layer{li}")
            for bi, blk in enumerate(layer):
                pre = f"layer{li}.{bi}"
                if isinstance(blk, Bottleneck):
                    c1 = self._conv(f"{pre}.conv1", blk.conv1, h, w)
                    c2 = self._conv(f"{pre}.conv2", blk.conv2, c1.OH, c1.OW)
                    c3 = self._conv(f"{pre}.conv3", blk.conv3, c2.OH, c2.OW)
                    convs = [c1, c2, c3]
                    bns = [BNL(f"{pre}.bn1", blk.bn1, blk.bn1.num_features),
                           BNL(f"{pre}.bn2", blk.bn2, blk.bn2.num_features),
                           BNL(f"{pre}.bn3", blk.bn3, blk.bn3.num_features)]
                    kind = "bottleneck"
                    ds = blk.downsample
                elif isinstance(blk, (BasicBlock, CifarBlock)):
                    c1 = self._conv(f"{pre}.conv1", blk.conv1, h, w)
                    c2 = self._conv(f"{pre}.conv2", blk.conv2, c1.OH, c1.OW)
                    convs = [c1, c2]
                    bns = [BNL(f"{pre}.bn1", blk.bn1, blk.bn1.num_features),
                           BNL(f"{pre}.bn2", blk.bn2, blk.bn2.num_features)]
                    kind = "basic"
                    ds = blk.downsample if isinstance(blk, BasicBlock) else (
                        blk.skip_connection if len(blk.skip_connection) > 0 else None)
                else:
                    raise TypeError(f"unsupported block {type(blk).__name__}")
                dsc = dsb = None
                if ds is not None:
                    dsc = self._conv(f"{pre}.downsample.0", ds[0], h, w)
                    dsb = BNL(f"{pre}.downsample.1", ds[1], ds[1].num_features)
                last = convs[-1]
                blk_l = BlockL(kind, convs, bns, dsc, dsb, (h, w, c), (last.OH, last.OW, last.OC))
                self.blocks.append(blk_l)
                h, w, c = last.OH, last.OW, last.OC
        self.feat_hw = (h, w)
        self.feat_c = c
        self.fc: nn.Linear = m.fc
        self.num_classes = m.fc.out_features
        self.convs: List[ConvL] = [self.stem] + [cv for b in self.blocks for cv in (b.convs + ([b.ds_conv] if b.ds_conv else []))]
        self.bns: List[BNL] = [self.stem_bn] + [bn for b in self.blocks for bn in (b.bns + ([b.ds_bn] if b.ds_bn else []))]
        for cv in self.convs[1:]:
            if cv.IC % 64 or cv.OC % 64:
                raise TypeError(f"{cv.name}: channels must be multiples of 64 for the HIP conv kernels")

    def _alloc_params(self):
        """Flat fp32 master / grad buffers; re-point module parameters at views of master."""
        dev = self.dev
        entries: List[Tuple[str, object, str, int]] = []  # (kind, obj, attr, numel)
        # Flat order = backward-segment order reversed (stem, layer1..4, fc): every backward
        # segment's gradients form ONE contiguous range -> one bucket, no gather/scatter.
        groups = [("conv1.", "bn1.")] + [(f"layer{i}.",) for i in range(1, 5)]
        for pre in groups:
            for cv in self.convs:
                if cv.name.startswith(pre) or (cv.stem and "conv1." in pre):
                    entries.append(("conv", cv, "weight", cv.numel))
            for bn in self.bns:
                if bn.name.startswith(pre) or (bn is self.stem_bn and "bn1." in pre):
                    entries.append(("bn_w", bn, "weight", bn.C))
                    entries.append(("bn_b", bn, "bias", bn.C))
        entries.append(("fc_w", self.fc, "weight", self.fc.weight.numel()))
        entries.append(("fc_b", self.fc, "bias", self.fc.bias.numel()))
        assert len(entries) == len(self.convs) + 2 * len(self.bns) + 2, "parameter grouping lost a tensor"
        # 16-element alignment of every tensor (vectorised kernels, 64-B bucket edges); every
        # backward segment's group (stem | layer1..4 | fc) starts on a multiple of param_align
        A = self.param_align
        group_of = []  # group index per entry (fc: its own group: the "head" backward segment)
        for gi, pre in enumerate(groups):
            for cv in self.convs:
                if cv.name.startswith(pre) or (cv.stem and "conv1." in pre):
                    group_of.append(gi)
            for bn in self.bns:
                if bn.name.startswith(pre) or (bn is self.stem_bn and "bn1." in pre):
                    group_of += [gi, gi]
        group_of += [len(groups), len(groups)]
        total = 0
        offs = []
        for i, e in enumerate(entries):
            if i > 0 and group_of[i] != group_of[i - 1]:
                total = (total + A - 1) // A * A
            offs.append(total)
            total += (e[3] + 15) // 16 * 16
        total = (total + A - 1) // A * A
        self.n_params = total
        self.master = torch.zeros(total, device=dev, dtype=torch.float32)
        self.grad = torch.zeros(total, device=dev, dtype=torch.float32)
        self.param_ranges: List[Tuple[str, int, int]] = []  # (param name, off, numel) for bucketing
        nbt_vals: List[int] = []
        nbt_mods: List[nn.BatchNorm2d] = []
        with torch.no_grad():
            for (kind, obj, attr, n), off in zip(entries, offs):
                if kind == "conv":
                    cv: ConvL = obj
                    cv.off = off
                    src = cv.mod.weight.detach().to(dev, torch.float32)  # [K, C, R, S]
                    flat = self.master[off:off + n]
                    flat.copy_(src.permute(0, 2, 3, 1).reshape(-1))
                    view = flat.view(cv.OC, cv.R, cv.S, cv.IC).permute(0, 3, 1, 2)  # channels_last view
                    _repoint(cv.mod.weight, view)
                    cv.grad = self.grad[off:off + n].view(cv.OC, cv.R * cv.S * cv.IC)
                    self.param_ranges.append((cv.name + ".weight", off, n))
                elif kind in ("bn_w", "bn_b"):
                    bn: BNL = obj
                    mod = bn.mod
                    p = getattr(mod, attr)
                    flat = self.master[off:off + n]
                    flat.copy_(p.detach().to(dev, torch.float32))
                    _repoint(p, flat)
                    if kind == "bn_w":
                        bn.off_w, bn.gamma, bn.dgamma = off, flat, self.grad[off:off + n]
                    else:
                        bn.off_b, bn.beta, bn.dbeta = off, flat, self.grad[off:off + n]
                    self.param_ranges.append((f"{bn.name}.{attr}", off, n))
                    # running stats stay module buffers (moved to device, updated in place)
                    mod.running_mean.data = mod.running_mean.data.to(dev, torch.float32)
                    mod.running_var.data = mod.running_var.data.to(dev, torch.float32)
                    if kind == "bn_w" and mod.num_batches_tracked is not None:
                        # one int64 counter per BN, all views of self.nbt (one add per step)
                        nbt_vals.append(int(mod.num_batches_tracked))
                        nbt_mods.append(mod)
                else:
                    p = getattr(self.fc, attr)
                    flat = self.master[off:off + n]
                    flat.copy_(p.detach().reshape(-1).to(dev, torch.float32))
                    view = flat.view(p.shape)
                    _repoint(p, view)
                    if attr == "weight":
                        self.fc_w_off, self.fc_w_grad = off, self.grad[off:off + n].view(p.shape)
                    else:
                        self.fc_b_off, self.fc_b_grad = off, self.grad[off:off + n]
                    self.param_ranges.append((f"fc.{attr}", off, n))
        self.param16 = torch.zeros(total, device=dev, dtype=torch.bfloat16) if self._want_param16 else None
        self.nbt = torch.tensor(nbt_vals, dtype=torch.int64, device=dev)
        for i, mod in enumerate(nbt_mods):
            mod.num_batches_tracked.data = self.nbt[i]
        # bf16 compute copies: KRSC fwd + CRSK dgrad per conv, fc weight
        n16 = 0
        descs = []
        for cv in self.convs:
            if cv.stem:
                continue
            fwd_off = n16
            n16 += cv.numel
            tr_off = n16
            n16 += cv.numel
            descs.append((cv.off, fwd_off, tr_off, cv.OC, cv.R * cv.S, cv.IC))
            cv._w16_off, cv._wt16_off = fwd_off, tr_off
        fc_off = n16
        n16 += self.fc.weight.numel()
        descs.append((self.fc_w_off, fc_off, -1, self.num_classes, 1, self.fc.in_features))
        # the stem's (K, 8, 8, 4) zero-padded copy and the fc bias: in the same buffer, same launch
        al = lambda v: (v + 63) // 64 * 64  # noqa: E731
        st = self.stem
        stem_off = n16 = al(n16)
        n16 += st.OC * 256
        descs.append((st.off, stem_off, -2, st.OC, st.R * 16 + st.S, st.IC))
        fcb_off = n16 = al(n16)
        n16 += self.num_classes
        descs.append((self.fc_b_off, fcb_off, -1, self.num_classes, 1, 1))
        self.w16buf = torch.zeros(al(n16) + 64, device=dev, dtype=torch.bfloat16)
        for cv in self.convs:
            if cv.stem:
                cv.w16 = self.w16buf[stem_off:stem_off + cv.OC * 256].view(cv.OC, 256)
                continue
            cv.w16 = self.w16buf[cv._w16_off:cv._w16_off + cv.numel].view(cv.OC, -1)
            cv.wt16 = self.w16buf[cv._wt16_off:cv._wt16_off + cv.numel].view(cv.IC, -1)
        self.fc_w16 = self.w16buf[fc_off:fc_off + self.fc.weight.numel()].view(self.num_classes, -1)
        self.fc_b16 = self.w16buf[fcb_off:fcb_off + self.num_classes]
        self._wdescs = descs  # + the per-step entries (_pack_step_descs, after the activations exist)
        self.wdesc = self._pack_wdesc(descs)
        self.n_wdesc = len(descs)
        self.stem_grad_tmp = torch.zeros(self.stem.OC, 256, device=dev, dtype=torch.float32)

    def _alloc_activations(self):
        N, dev, bf = self.N, self.dev, torch.bfloat16
        E = lambda *s: torch.empty(*s, device=dev, dtype=bf)  # noqa: E731
        st = self.stem
        self.x4 = torch.zeros(N, self.H, self.W, 4, device=dev, dtype=bf)
        self.y0 = E(N, st.OH, st.OW, st.OC)
        ph, pw = self.pool_hw
        self.p0 = E(N, ph, pw, st.OC)
        self.parg = torch.empty(N, ph, pw, st.OC, device=dev, dtype=torch.uint8)
        self.dp0 = E(N, ph, pw, st.OC)
        # pooled-gradient buffer only for pool geometries the fused stem backward does not cover
        self.da0 = None if K.pool_bn_bwd_supported(st.OC, self.pool_k, self.pool_s) else E(N, st.OH, st.OW, st.OC)
        # pre-BN stem value at each pool argmax (training): the stem BN-backward reduction runs over
        # the pooled positions instead of gathering over the full-resolution stem output
        self.pymax = E(N, ph, pw, st.OC) if self.da0 is None and self.pool_reduce else None
        self.dy0 = E(N, st.OH, st.OW, st.OC)
        wsmax = 0
        for b in self.blocks:
            b.ys = [E(N, cv.OH, cv.OW, cv.OC) for cv in b.convs]
            b.dys = [E(N, cv.OH, cv.OW, cv.OC) for cv in b.convs]
            b.das = [E(N, cv.OH, cv.OW, cv.OC) for cv in b.convs[:-1]]
            # BN outputs inside the block (inputs of convs 1..n-1), written in backward by the MASK_Y
            # dgrad epilogue that computes them for the ReLU mask anyway: the weight gradient then
            # reads them instead of re-applying BN+ReLU to every staged tile
            b.acts = [E(N, cv.OH, cv.OW, cv.OC) if self.act_writeback else None for cv in b.convs[:-1]]
            # acts[j] computed in the forward (eight-wave consumer conv j+1): see self.fast_mat
            b.mat = [self._materialize(b.convs[j + 1]) and b.acts[j] is not None for j in range(len(b.convs) - 1)]
            h, w, c = b.in_shape
            b.dx = E(N, h, w, c)
            if b.ds_conv is not None:
                dcv = b.ds_conv
                if dcv.R != 1 or dcv.S != 1 or dcv.pad != 0:
                    raise TypeError(f"{dcv.name}: downsample must be a 1x1 pad-0 conv")
                b.yd = E(N, dcv.OH, dcv.OW, dcv.OC)
                b.dyd = E(N, dcv.OH, dcv.OW, dcv.OC)
                b.dsbuf = E(N, dcv.OH, dcv.OW, dcv.IC)  # dense dgrad of the strided 1x1
            oh, ow, oc = b.out_shape
            b.out = E(N, oh, ow, oc)
            # 1-bit ReLU mask of the block output (the next block's dgrad epilogue masks with it:
            # 1/16 of the bytes of re-reading the bf16 output)
            b.obits = torch.empty(N * oh * ow * oc // 8, device=dev, dtype=torch.uint8)
        for cv in self.convs:
            ktot = 256 if cv.stem else cv.R * cv.S * cv.IC
            wsmax = max(wsmax, cv.OC * ktot)
        # split-K wgrad workspace: up to 64 splits of the largest layer, >= 64 MiB
        self.ws = torch.empty(max(64 * wsmax, 16 << 20), device=dev, dtype=torch.float32)
        # The step's exposed end (tools/step_timeline.py): after the last data gradient only the side
        # stream's last batch (layer1's weight gradients) and the stem weight gradient behind it run.
        # Small steps (< 0.5 TFLOP of forward conv work) run the stem weight gradient on the main stream
        # beside that batch (stem_wg_main; CIFAR 257.0-257.6k vs 252.1-253.8k, TinyImageNet 96.7-96.8k
        # vs 96.0-96.1k img/s; the b1024 headline loses 0.3 %: 16.48-16.49k vs 16.53-16.55k), and the
        # TinyImageNet class (50-500 GFLOP) also moves the batch's last two gradients to the main
        # stream's end (tail_main, their own workspace of ws's size: the same split depths, the same
        # bits): 97.5-97.8k img/s; CIFAR loses with it (profiles/r5_tail/)
        fl = self.fwd_flops
        cfg, pol = self.cfg, self.cfg.policy
        # side_defer: launch each side batch after the main stream's next kernel (see _flush_side).
        # Default: on for the small steps (< 0.5 TFLOP of forward conv work: CIFAR +0.7 %, TinyImageNet
        # neutral), off for the b1024 headline (-0.4 % / neutral); the multi-rank one-graph step turns it
        # on (its collectives ride the side stream: TinyImageNet +2.8 %, CIFAR +5 %, profiles/r5_side_defer/)
        self.side_defer = cfg.side_defer if cfg.side_defer is not None else (pol.small(fl) or self.side_block)
        # side_cu_reserve: side-stream weight gradients sized to one round over all but N CUs, so
        # the main chain's small kernels find a CU (the BN-backward coefficient launches took 4.9 us alone
        # and 26.5 us beside the weight gradients); default 128 from the TinyImageNet class up (64: headline
        # +0.8 %, TinyImageNet +0.6-0.9 %; re-swept with the per-block forks and main-stream tails, 128 over
        # 64: TinyImageNet +1.8 %, headline +0.4 %; 160+ loses), 0 for the CIFAR class (64: -0.4 %, 128:
        # -1 %): profiles/r5_cu_reserve/
        self.side_cu_reserve = (cfg.side_cu_reserve if cfg.side_cu_reserve is not None
                                else (0 if pol.tiny(fl) else 128))
        # (with the per-block forks from 500 GFLOP up, together with two of the last block's weight
        # gradients: headline +0.38 % over five interleaved rounds, profiles/r5_side_defer/block_tail.txt)
        self.stem_wg_main = cfg.stem_wg_main if cfg.stem_wg_main is not None else (pol.small(fl) or self.side_block)
        # (with the deferred launch the TinyImageNet class moves three: 99.7-100.4k vs 99.0-99.6k img/s)
        self.tail_main = (cfg.tail_main if cfg.tail_main is not None
                          else ((3 if self.side_defer else 2) if pol.mid(fl) else 0))
        # the fused conv3 backward's persistent grid spans only this many CUs, so the side stream's weight
        # gradients keep theirs (dwf_cus; 0 = all): TinyImageNet class 128 (+0.3 %), the headline
        # loses with any span (-0.9 % at 192), profiles/r5_side_defer/tiny_knobs_late.txt
        self.dwf_cus = cfg.dwf_cus if cfg.dwf_cus is not None else (128 if pol.mid(fl) else 0)
        # the same as tail_main for the per-block side forks (overlap_wgrad 3): the last block's
        # last N weight gradients (TinyImageNet at the 128-CU reservation: 2 over 1 +0.4 % in five of five
        # interleaved rounds; headline +0.38 % with the stem's, profiles/r5_side_defer/block_tail.txt)
        self.block_tail_main = cfg.block_tail_main
        self._main_tail = []
        self._join_evt = None
        # set by the multi-rank trainer when its collectives share the side stream (comm_side):
        # every segment join then waits for the event behind the segment's batch, not for the
        # collectives queued behind it on the same stream (the final join waits for everything)
        self.event_joins = False
        # the downsample conv's forward beside conv2 / conv3 on the side stream: +0.24 % on the headline
        # over five interleaved rounds, TinyImageNet neutral alone and +0.67 % with its block tail of one,
        # CIFAR +0.6 % (profiles/r5_side_defer/ds_fwd.txt, block_tail.txt, cifar_late.txt)
        self.ds_fwd_side = cfg.ds_fwd_side
        # lazy_join: no intermediate joins of the batched side stream -- every side batch reads only
        # its own segment's per-block buffers (never reused within a step) and the workspaces of the main
        # stream's weight gradients are separate, so only the final join (before the optimizer) orders
        # the two; not with collectives on their own stream (they wait on the main stream at the joins)
        # (default: the CIFAR class, < 50 GFLOP of forward conv work, +1.2 %; TinyImageNet -0.3 %, the
        # headline -0.5 %: profiles/r5_side_defer/lazy_join.txt)
        self.lazy_join = cfg.lazy_join if cfg.lazy_join is not None else (pol.tiny(fl) or self.side_block)
        self._pending_side = []
        # the stem weight gradient's own slabs when it runs on the main stream (its split count depends
        # on the grid, not on the workspace capacity)
        self.ws_stem = (torch.empty(40 << 20, device=dev, dtype=torch.float32)
                        if dev.type == "cuda" and self.stem_wg_main else self.ws)
        # (not tied to the batched layout: the multi-rank trainer may switch a per-block default back to it)
        self.ws_main = (torch.empty_like(self.ws) if ((self.tail_main > 0 or self.block_tail_main > 0)
                                                      and dev.type == "cuda"
                                                       and self.overlap_wgrad) else self.ws)
        # the fused conv3 backward runs on the main stream while side-stream weight gradients use
        # self.ws: its per-workgroup slabs get their own workspace (<= 1024 slabs + 64 partials)
        fused = [b.convs[-1] for i, b in enumerate(self.blocks) if self._fuse3(b, i == len(self.blocks) - 1)]
        # (slab count = resident workgroups, K.dwfused_grid; the CPU reference path uses no workspace)
        self.ws_dw = (torch.empty((max((K.dwfused_grid(c.IC, c.OC) + 64) * c.OC * c.IC for c in fused)
                                   if dev.type == "cuda" else 16), device=dev, dtype=torch.float32)
                      if fused else None)
        fh, fw = self.feat_hw
        self.dfeat = self.blocks[-1].out  # placeholder name; real grad buffer below
        self.dlast = E(N, fh, fw, self.feat_c)
        self.g_last = E(N, fh, fw, self.feat_c)
        self.pooled = E(N, self.feat_c)
        self.dpooled = E(N, self.feat_c)
        self.logits = E(N, self.num_classes)
        self.dlogits = E(N, self.num_classes)
        # split-K partials of the head GEMMs (K.head_splitk: the few-tile, long-K fc shapes)
        self.head_ws = (torch.empty(8 * max(N * self.num_classes, self.num_classes * self.feat_c), device=dev,
                                    dtype=torch.float32) if dev.type == "cuda" else None)
        self.labels = torch.zeros(N, device=dev, dtype=torch.int64)
        sh, sw = self.src_hw
        self.img_u8 = torch.zeros(N, sh, sw, 3 if self.in_ch != 1 else 1, device=dev, dtype=torch.uint8)
        self.boxes = torch.tensor([[0.0, 0.0, float(sh), float(sw)]] * N, device=dev)  # full-image default
        self.flip = torch.zeros(N, device=dev, dtype=torch.uint8)
        self.metrics = torch.zeros(2, device=dev, dtype=torch.float64)  # loss sum, correct (fp64 atomics)
        # BN state arena
        # fp64 statistics slabs, contiguous: zeroed by ONE memset per step
        ns = self.nshard
        self.stats_region = torch.zeros(sum(2 * 2 * ns * bn.C for bn in self.bns), device=dev, dtype=torch.float64)
        o = 0
        for bn in self.bns:
            bn.stats = self.stats_region[o:o + 2 * ns * bn.C]
            o += 2 * ns * bn.C
            bn.bstats = self.stats_region[o:o + 2 * ns * bn.C]
            o += 2 * ns * bn.C
        self.bn_arena = torch.zeros(sum(7 * bn.C for bn in self.bns), device=dev, dtype=torch.float32)
        o = 0
        for bn in self.bns:
            bn.scale = self.bn_arena[o:o + bn.C]; o += bn.C
            bn.shift = self.bn_arena[o:o + bn.C]; o += bn.C
            bn.mean = self.bn_arena[o:o + bn.C]; o += bn.C
            bn.invstd = self.bn_arena[o:o + bn.C]; o += bn.C
            bn.coeff = self.bn_arena[o:o + 3 * bn.C]; o += 3 * bn.C
        self.mean_t = torch.tensor(IMAGENET_MEAN)
        self.std_t = torch.tensor(IMAGENET_STD)
        # CutMix state (enable_cutmix): sampled on the host per step, consumed on the device by the
        # augment kernel (box paste) and the CE kernel (mixed soft targets)
        self.cutmix = False
        self.mix_perm = self.mix_box = self.mix_lam = self.labels2 = None

    def _pack_wdesc(self, descs) -> torch.Tensor:
        # WDesc {long long src, fwd, tr; int K, RS, C, pad} = 40 bytes
        raw = []
        for (src, f, t, k, rs, c) in descs:
            raw.append(torch.tensor([src, f, t], dtype=torch.int64).view(torch.int32))
            raw.append(torch.tensor([k, rs, c, 0], dtype=torch.int32))
        return torch.cat(raw).to(self.dev)

    def _pack_step_descs(self) -> None:
        """The training step's weight-prep launch also zeroes the BN statistics slabs and counts
        num_batches_tracked (prepare_weights(step=True))."""
        extra = [(self.stats_region.data_ptr(), 0, -3, self.stats_region.numel(), 0, 0)]
        if self.nbt.numel():
            extra.append((self.nbt.data_ptr(), 0, -4, self.nbt.numel(), 0, 0))
        self.wdesc_step = self._pack_wdesc(self._wdescs + extra) if self.dev.type == "cuda" else None
        self.n_wdesc_step = len(self._wdescs) + len(extra)
        self._stats_zeroed = False

    def build_fins(self) -> None:
        """(Re)build every BN's finalize descriptors (K.BnFin: raw pointers to its statistics, affine
        parameters, running stats and outputs) -- again whenever one of those tensors is reallocated."""
        N = self.N
        pairs = [(self.stem_bn, self.stem)]
        for b in self.blocks:
            pairs += list(zip(b.bns, b.convs))
            if b.ds_conv is not None:
                pairs.append((b.ds_bn, b.ds_conv))
        for bn, cv in pairs:
            mod = bn.mod
            cnt = N * cv.OH * cv.OW
            mom = mod.momentum if mod.momentum is not None else 0.1
            bn.fin_f = bn.fin_b = None
            if bn.C % 64:
                continue
            bn.fin_f = K.BnFin(K.BnFin.FWD, bn.stats, cnt, gamma=bn.gamma, beta=bn.beta, eps=mod.eps,
                               momentum=mom if mod.track_running_stats else 0.0, running_mean=mod.running_mean,
                               running_var=mod.running_var, scale=bn.scale, shift=bn.shift, mean=bn.mean,
                               invstd=bn.invstd)
            bn.fin_b = K.BnFin(K.BnFin.BWD, bn.bstats, cnt, gamma=bn.gamma, mean=bn.mean, invstd=bn.invstd,
                               coeff=bn.coeff, dgamma=bn.dgamma, dbeta=bn.dbeta)
        for b in self.blocks:  # the tail prologue's [block BN, shortcut BN] descriptor arrays, up front
            if b.ds_bn is not None and b.bns[-1].fin_f is not None and b.ds_bn.fin_f is not None:
                if b.bns[-1].fin_f.desc is not None and b.ds_bn.fin_f.desc is not None:
                    b.bns[-1].fin_f.pair_ptr(b.ds_bn.fin_f)

    def _ff(self, bn):
        """The forward finalize descriptor to hand the conv producing ``bn``'s statistics (training)."""
        return bn.fin_f if self.training and self.fuse_fin else None

    def _fused_fin(self, bn) -> bool:
        return self.fuse_fin and bn.fin_f is not None

    def enable_cutmix(self) -> None:
        dev = self.dev
        self.cutmix = True
        self.mix_perm = torch.arange(self.N, device=dev, dtype=torch.int32)
        self.mix_box = torch.zeros(4, device=dev, dtype=torch.int32)  # y0, y1, x0, x1 (empty: no mixing)
        self.mix_lam = torch.ones(1, device=dev, dtype=torch.float32)
        self.labels2 = torch.zeros(self.N, device=dev, dtype=torch.int64)

    # ----------------------------------------------------------------------------------
    # per-step pieces
    # ----------------------------------------------------------------------------------
    def prepare_weights(self, step: bool = False):
        """fp32 master -> bf16 compute copies (KRSC fwd, CRSK dgrad, fc weight and bias, stem 8x8x4),
        one launch. ``step``: a training step follows -- the same launch zeroes the BN statistics and
        counts num_batches_tracked (the forward then skips its own zeroing)."""
        src = self.master if self.param16 is None else self.param16  # ZeRO: the all-gathered bf16 copy
        if step and self.wdesc_step is not None:
            K.weight_prep(src, self.w16buf, self.wdesc_step, self.n_wdesc_step)
            self._stats_zeroed = True
            return
        K.weight_prep(src, self.w16buf, self.wdesc, self.n_wdesc)
        if step:
            self.nbt.add_(1)

    def bn_param_blocks(self) -> List[Tuple[int, int]]:
        """Contiguous [lo, hi) blocks of the flat buffer holding BatchNorm affine parameters (read in
        fp32 by the BN kernels), merged where adjacent."""
        rs = sorted((o, o + (bn.C + 15) // 16 * 16) for bn in self.bns for o in (bn.off_w, bn.off_b))
        out: List[Tuple[int, int]] = []
        for lo, hi in rs:
            if out and out[-1][1] == lo:
                out[-1] = (out[-1][0], hi)
            else:
                out.append((lo, hi))
        return out

    def load_input_u8(self, flip: Optional[torch.Tensor] = None):
        """uint8 images (+ per-sample crop boxes / flips in self.boxes / self.flip) -> bf16 NHWC4."""
        mean = self.norm_mean or (IMAGENET_MEAN if self.in_ch == 3 else (0.5, 0.5, 0.5))
        std = self.norm_std or (IMAGENET_STD if self.in_ch == 3 else (0.5, 0.5, 0.5))
        if self.norm_mean and len(mean) == 1:
            mean, std = mean * 3, std * 3
        mix = self.cutmix and self.training
        K.augment_u8(self.img_u8, self.x4, self.boxes, mean, std, self.flip if flip is None else flip,
                     perm=self.mix_perm if mix else None, mixbox=self.mix_box if mix else None)
        if mix:  # the pasted samples' labels (device gather, inside the captured step)
            torch.index_select(self.labels, 0, self.mix_perm.long(), out=self.labels2)

    def _bn_fwd(self, bn: BNL, count: int):
        mod = bn.mod
        if self.training:
            mom = mod.momentum if mod.momentum is not None else 0.1
            K.bn_finalize(bn.stats, count, bn.gamma, bn.beta, mod.eps, mom if mod.track_running_stats else 0.0,
                          mod.running_mean, mod.running_var, bn.scale, bn.shift, bn.mean, bn.invstd)
        else:
            K.bn_eval_coeff(bn.gamma, bn.beta, mod.eps, mod.running_mean, mod.running_var, bn.scale, bn.shift)

    def forward(self, smoothing: float = 0.0, compute_grad: bool = True, grad_scale: float = 1.0,
                metrics: bool = True, features_only: bool = False):
        """Full forward incl. loss. Assumes x4 / labels filled and prepare_weights() done.
        ``features_only``: stop after global average pooling and return ``self.pooled`` [N, C]
        (frozen-backbone feature extraction; the fc / loss are left to the caller)."""
        tr = self.training
        if tr and not self._stats_zeroed:
            self.stats_region.zero_()
        self._stats_zeroed = False
        N = self.N
        st, sbn = self.stem, self.stem_bn
        K.conv_stem_fwd(self.x4, st.w16, self.y0, R=st.R, S=st.S, stride=st.stride, pad=st.pad,
                        stats=sbn.stats if tr else None)
        sfin = sbn.fin_f if (tr and self.fin_in and sbn.fin_f is not None) else None  # (finalized by the pool)
        if sfin is None:
            self._bn_fwd(sbn, N * st.OH * st.OW)
        K.maxpool_fwd(self.y0, self.p0, self.parg, K=self.pool_k, stride=self.pool_s, pad=self.pool_p,
                      scale=sbn.scale, shift=sbn.shift, relu=True, ymax=self.pymax if tr else None, fin=sfin)
        x = self.p0
        # ds_fwd_side: a downsample conv reads only the block input (written by the block's conv1
        # tail prologue): it runs on the side stream beside conv2 / conv3, launched like a deferred side
        # batch after the main stream's next kernel, joined at the block's end
        ds_launch = {} if (self.ds_fwd_side and tr and self.dev.type == "cuda" and self.overlap_wgrad) else None
        pending = None  # previous block whose output this block's conv1 computes (tail prologue)
        out_fin = None  # the last BN's forward finalize, done by the block-output bn_apply (fin_in)
        for bi, b in enumerate(self.blocks):
            prev_bn = None
            deferred = None  # BN of conv i-1 whose finalize conv i's prologue performs (fin_in)
            for i, cv in enumerate(b.convs):
                if i == 0 and pending is not None:
                    pb, res, rsc, rsh, pfin, prfin = pending
                    K.conv_fwd(pb.ys[-1], cv.w16, b.ys[0], R=cv.R, S=cv.S, stride=cv.stride, pad=cv.pad,
                               stats=b.bns[0].stats if tr else None, in_scale=pb.bns[-1].scale,
                               in_shift=pb.bns[-1].shift, relu_in=True, tail_res=res, tail_res_scale=rsc,
                               tail_res_shift=rsh, tail_out=pb.out, tail_bits=pb.obits if tr else None,
                               fin=self._ff(b.bns[0]), fin_in=pfin, fin_in_res=prfin)
                    pending = None
                elif i > 0 and b.mat[i - 1]:  # materialised BN output -> plain-operand (eight-wave) conv
                    K.bn_apply(b.ys[i - 1], prev_bn.scale, prev_bn.shift, b.acts[i - 1], relu=True)
                    K.conv_fwd(b.acts[i - 1], cv.w16, b.ys[i], R=cv.R, S=cv.S, stride=cv.stride, pad=cv.pad,
                               stats=b.bns[i].stats if tr else None, fin=self._ff(b.bns[i]))
                else:
                    src = x if i == 0 else b.ys[i - 1]
                    K.conv_fwd(src, cv.w16, b.ys[i], R=cv.R, S=cv.S, stride=cv.stride, pad=cv.pad,
                               stats=b.bns[i].stats if tr else None,
                               in_scale=prev_bn.scale if prev_bn else None,
                               in_shift=prev_bn.shift if prev_bn else None, relu_in=True,
                               fin=self._ff(b.bns[i]), fin_in=deferred.fin_f if deferred is not None else None)
                deferred = None
                # (the fork follows conv1, whose tail prologue writes the block input; forking before
                # conv1 where the input is already in memory measured neutral in round 5)
                if i == 0 and ds_launch is not None and b.ds_conv is not None:
                    ds_launch[bi] = self._ds_fwd_on_side(b, x, N)
                nxt = self.blocks[bi + 1] if bi + 1 < len(self.blocks) else None
                c1 = nxt.convs[0] if nxt is not None else None
                tail = (self.fuse_tail and c1 is not None
                        and K.tail_supported(b.out_shape[2], c1.R, c1.S, c1.stride, c1.pad))
                if self._ff(b.bns[i]) is None:
                    if (tr and self.fin_in and i + 1 < len(b.convs) and not b.mat[i]
                            and b.bns[i].fin_f is not None):
                        deferred = b.bns[i]  # finalized by the next conv's prologue
                    elif tr and self.fin_in and i + 1 == len(b.convs) and b.bns[i].fin_f is not None:
                        out_fin = b.bns[i].fin_f  # finalized by the block-output bn_apply / next conv1 below
                    else:
                        self._bn_fwd(b.bns[i], N * cv.OH * cv.OW)
                prev_bn = b.bns[i]
            last = b.bns[-1]
            res_fin = None
            if b.ds_conv is not None:
                dc = b.ds_conv
                side_ds = ds_launch.get(bi) if ds_launch else None
                if side_ds is None:
                    K.conv_fwd(x, dc.w16, b.yd, R=dc.R, S=dc.S, stride=dc.stride, pad=dc.pad,
                               stats=b.ds_bn.stats if tr else None, fin=self._ff(b.ds_bn))
                if self._ff(b.ds_bn) is None:
                    if tr and self.fin_in and b.ds_bn.fin_f is not None:
                        res_fin = b.ds_bn.fin_f  # finalized by the block-output bn_apply / next conv1 below
                    elif side_ds is None:
                        self._bn_fwd(b.ds_bn, N * dc.OH * dc.OW)
                if side_ds is not None:  # (launched on the side stream after conv1: join it here)
                    self.launch_pending()
                    torch.cuda.current_stream(self.dev).wait_event(side_ds)
                res, rsc, rsh = b.yd, b.ds_bn.scale, b.ds_bn.shift
            else:
                res, rsc, rsh = x, None, None
            if tail:
                # b.out (+ its mask) is written by the next block's conv1 (which also finalizes the
                # tail BNs deferred above)
                pending = (b, res, rsc, rsh, out_fin, res_fin)
            else:
                K.bn_apply(b.ys[-1], last.scale, last.shift, b.out, res=res, res_scale=rsc, res_shift=rsh,
                           relu=True, mbits=b.obits if tr else None, fin=out_fin, res_fin=res_fin)
            out_fin = None
            x = b.out
        K.avgpool_fwd(x, self.pooled)
        if features_only:
            return self.pooled
        F, Cn = self.feat_c, self.num_classes
        K.small_gemm(self.pooled, self.fc_w16, self.logits, M=N, N=Cn, K=F, bias=self.fc_b16, ws=self.head_ws)
        mix = self.cutmix and self.training
        K.softmax_ce(self.logits, self.labels, self.dlogits if compute_grad else None, None,
                     self.metrics if metrics else None, smoothing=smoothing, grad_scale=grad_scale,
                     labels2=self.labels2 if mix else None, lam=self.mix_lam if mix else None)
        return self.logits

    def _ds_fwd_on_side(self, b, x, N):
        """Queue block b's downsample conv (+ its BN finalize unless a consumer does it) for the side
        stream, forked from the main stream's current point; returns the event that ends it."""
        dc, side = b.ds_conv, self.side_stream()
        fork, done = torch.cuda.Event(), torch.cuda.Event()
        fork.record(torch.cuda.current_stream(self.dev))

        def launch():
            side.wait_event(fork)
            with torch.cuda.stream(side):
                K.conv_fwd(x, dc.w16, b.yd, R=dc.R, S=dc.S, stride=dc.stride, pad=dc.pad, stats=b.ds_bn.stats,
                           fin=self._ff(b.ds_bn))
                if self._ff(b.ds_bn) is None and not (self.fin_in and b.ds_bn.fin_f is not None):
                    self._bn_fwd(b.ds_bn, N * dc.OH * dc.OW)
            done.record(side)
        if self._pending_side:  # (joined by its event at the block's end: no _side_pending)
            self._pending_side.append(launch)
        else:
            self._pending_side = [launch]
            K.set_post_launch(self.launch_pending)
        return done

    def backward_segments(self):
        """Yield closures, one per backward segment; after segment k all params whose
        names appear in ``segment_params[k]`` have final gradients (bucket-ready points)."""
        return self._segments

    def build_backward(self):
        segs = []
        # head + layer4 blocks, each stage its own segment (reverse order)
        stages: Dict[int, List[int]] = {}
        bi = 0
        for li in range(1, 5):
            n = len(getattr(self.model, f"layer{li}"))
            stages[li] = list(range(bi, bi + n))
            bi += n
        segs.append(("head", self._bwd_head))
        for li in (4, 3, 2, 1):
            idx = list(reversed(stages[li]))
            segs.append((f"layer{li}", (lambda idx=idx, li=li: [
                (self._bwd_block(i), self._block_flush(li == 1 and j == len(idx) - 1))
                for j, i in enumerate(idx)])))
        segs.append(("stem", self._bwd_stem))
        # every segment ends with its weight gradients complete on the main stream (join)
        last = len(segs) - 1
        self._segments = [(n, (lambda fn=fn, k=k: (fn(), self._join_side(final=k == last,
                                                                         tail_main=k == last - 1))))
                          for k, (n, fn) in enumerate(segs)]
        return self._segments

    # --------------------------------------------------------------------------------------
    # wgrad overlap: a conv's weight gradient depends only on its dY and X, not on the dgrad
    # chain, so it runs on a side stream while the main stream continues with the (memory-bound)
    # dgrad epilogue / BN-backward kernels of the same and next layers. Forked and joined with
    # stream waits, which HIP-graph capture records as parallel branches of the step graph.
    # (Measured +0.4 % in graphs, +1 % eager at batch 1024: every launch already fills the GPU.)
    def _side(self, fn):
        if self.dev.type != "cuda" or not self.overlap_wgrad:
            fn()
            return
        if self.side_batch or self.side_block:  # launched as one batch (_flush_side)
            self._side_q.append(fn)
            return
        if self._wstream is None:
            self._wstream = torch.cuda.Stream(device=self.dev)
        self._wstream.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(self._wstream):
            fn()
        self._side_pending = True

    def _wgrad(self, *args, **kw):
        if self.side_cu_reserve and self.dev.type == "cuda" and self.overlap_wgrad:
            kw["cu_reserve"] = self.side_cu_reserve  # one round over all but N CUs (side_cu_reserve)
        # (a queued weight gradient takes the batch's deferred-reduction list when it is launched)
        # (ws: the workspace override of a gradient moved to the main stream's tail, see _join_side)
        self._side(lambda batch=None, ws=None: K.conv_wgrad(*args[:3], args[3] if ws is None else ws, *args[4:],
                                                          defer=batch, **kw))

    def _flush_side(self, join_evt: Optional[torch.cuda.Event] = None) -> bool:
        """Fork the side stream once from the main stream and launch the queued weight gradients on it
        (``join_evt``: recorded on the side stream right behind them). With ``side_defer`` the fork point
        is an event recorded on the main stream now and the launch waits for the main stream's next
        kernel launch (kernels.set_post_launch): in the captured graph the fork node's FIRST edge then
        continues the main chain, so the runtime's depth-first split of the graph into per-queue lists
        keeps the main chain in one list and chains the side batches into another."""
        if not self._side_q:
            return False
        self.launch_pending()  # (at most one deferred batch)
        if self._wstream is None:
            self._wstream = torch.cuda.Stream(device=self.dev)
        q = self._side_q
        self._side_q = []
        self._side_pending = True
        main = torch.cuda.current_stream(self.dev)
        fork = None
        if self.side_defer:
            fork = torch.cuda.Event()
            fork.record(main)
        else:
            self._wstream.wait_stream(main)

        def launch():
            if fork is not None:
                self._wstream.wait_event(fork)
            # (each batch of a step takes an arena region of its own)
            batch = K.ReduceBatch(self.wred_arena, self._wred_off) if self.defer_reduce else None
            with torch.cuda.stream(self._wstream):
                for fn in q:
                    if batch is not None and getattr(fn, "__defaults__", None):
                        fn(batch)  # a weight gradient that can defer its reduction
                    else:
                        fn()
                if batch is not None:
                    batch.flush()
            if join_evt is not None:
                join_evt.record(self._wstream)
            if batch is not None:
                # (the next batch starts past everything this one asked for, placed or not: a warm-up
                # step that found the arena too small then sizes it for the whole step at once)
                self._wred_off = batch.need
                if batch.need > self.wred_arena.numel() and not torch.cuda.is_current_stream_capturing():
                    # grown for the next steps (the eager warm-up steps size it before any capture)
                    torch.cuda.current_stream(self.dev).wait_stream(self._wstream)
                    self.wred_arena = torch.empty(batch.need, device=self.dev, dtype=torch.float32)

        if fork is None:
            launch()
        else:
            self._pending_side = [launch]
            K.set_post_launch(self.launch_pending)
        return True

    def defer_on_side(self, fn) -> bool:
        """Queue ``fn`` (run under the side stream) behind the deferred batch; False: nothing deferred."""
        if not self._pending_side:
            return False

        def run():
            with torch.cuda.stream(self._wstream):
                fn()
        self._pending_side.append(run)
        return True

    def launch_pending(self) -> None:
        """Launch the deferred side batch (and what was queued behind it) now."""
        if not self._pending_side:
            return
        items = self._pending_side
        self._pending_side = []
        K.set_post_launch(None, owner=self.launch_pending)
        for f in items:
            f()

    def drop_pending(self) -> None:
        """Forget a deferred side batch (the step that queued it failed)."""
        self._pending_side = []
        K.set_post_launch(None, owner=self.launch_pending)

    def _block_flush(self, last: bool = False):
        if self.side_block and self.dev.type == "cuda" and self.overlap_wgrad:
            # the step's last block: its last block_tail_main weight gradients run on the main stream after
            # the stem's backward (their own workspace) instead of behind the rest on the side stream
            n = self.block_tail_main if last else 0
            if n > 0 and len(self._side_q) > n:
                self._main_tail = self._side_q[-n:]
                self._side_q = self._side_q[:-n]
            self._flush_side()  # this block's weight gradients, under the next block's data gradients

    def side_stream(self):
        """The weight-gradient side stream (created on first use)."""
        if self._wstream is None:
            self._wstream = torch.cuda.Stream(device=self.dev)
        return self._wstream

    def _join_side(self, final: bool = True, tail_main: bool = False):
        if self.side_batch and self.dev.type == "cuda" and self.overlap_wgrad:
            # batched side stream: the segment's weight gradients fork ONCE, after its data gradients,
            # and run under the NEXT segment's backward; joined one segment later (at most one batch in
            # flight: they share self.ws) and at the end of the backward
            if self._main_tail:
                # the previous batch's tail (moved off the side stream at the previous join) on the main
                # stream, after this segment's data gradients, beside the batch's head on the side stream
                for fn in self._main_tail:
                    fn(None, self.ws_main)
                self._main_tail = []
            self.launch_pending()
            if self._side_pending and self.lazy_join and not final:
                pass  # (lazy_join: the final join below waits for everything)
            elif self._side_pending:
                if self._join_evt is not None:  # the previous batch only, not the blocks flushed since
                    torch.cuda.current_stream(self.dev).wait_event(self._join_evt)
                    self._side_pending = self.event_joins  # (collectives behind it)
                else:
                    torch.cuda.current_stream(self.dev).wait_stream(self._wstream)
                    self._side_pending = False
            self._join_evt = None
            # the LAST batch (layer1) is exposed at the end of the step: only the stem's short backward
            # runs beside it -- its last tail_main gradients go to the main stream's end instead
            # (their own workspace)
            n = self.tail_main if tail_main else 0
            if n > 0 and len(self._side_q) > n:
                self._main_tail = self._side_q[-n:]
                self._side_q = self._side_q[:-n]
            want = self.event_joins and not final
            evt = torch.cuda.Event() if want else None
            if self._flush_side(join_evt=evt):
                self._join_evt = evt
            elif want and self._side_pending:
                self._join_evt = torch.cuda.Event()
                self._join_evt.record(self._wstream)
            if not final:
                return
        elif self.side_block and self.dev.type == "cuda" and self.overlap_wgrad:
            self._flush_side()  # (the stem / head segments queue theirs here), joined below
            if self.lazy_join and not final:
                return  # (lazy_join: per-block batches too, joined only at the end)
            if final and self._main_tail:
                for fn in self._main_tail:  # (see _block_flush)
                    fn(None, self.ws_main)
                self._main_tail = []
        self.launch_pending()
        if self._side_pending:
            torch.cuda.current_stream(self.dev).wait_stream(self._wstream)
            self._side_pending = False
        self._wred_off = 0  # (every batch of the step has been joined)

    def _bwd_head(self):
        # fc on MFMA (csrc/head_ops.hip): dW = dlogits^T pooled (fp32, straight into the flat gradient),
        # db = column sums of dlogits, dpooled = dlogits W
        N, F, Cn = self.N, self.feat_c, self.num_classes
        K.small_gemm(self.dlogits, self.pooled, self.fc_w_grad, ta=True, tb=True, M=Cn, N=F, K=N, ws=self.head_ws)
        K.colsum(self.dlogits, self.fc_b_grad)
        K.small_gemm(self.dlogits, self.fc_w16, self.dpooled, ta=False, tb=True, M=N, N=F, K=Cn, ws=self.head_ws)
        K.avgpool_bwd(self.dpooled, self.dlast)

    def _cin(self, bn, count=None) -> bool:
        """Does ``bn``'s next BN-backward apply pass finalize the coefficients inside its launch
        (coeff_in: no bn_bwd_coeff launch in front of it)?"""
        f = bn.fin_b
        return (self.coeff_in and f is not None and f.desc is not None
                and (self.coeff_in_maxc is None or bn.C <= self.coeff_in_maxc)
                and (count is None or float(count) == f.count))

    def _coeff(self, bn, count) -> None:
        """The standalone backward finalize of ``bn`` (its consumer needs ``bn.coeff`` in memory)."""
        K.bn_bwd_coeff(bn.bstats, count, bn.gamma, bn.mean, bn.invstd, bn.coeff, bn.dgamma, bn.dbeta)

    def _bn_bwd(self, bn: BNL, dout, y, dy, count, mask_mode, mref=None, gout=None):
        K.bn_bwd_reduce(dout, y, bn.mean, bn.invstd, bn.bstats, mask_mode=mask_mode, mref=mref,
                        scale=bn.scale, shift=bn.shift)
        fin = bn.fin_b if self._cin(bn, count) else None
        if fin is None:
            self._coeff(bn, count)
        K.bn_bwd_apply(dout, y, bn.coeff, dy, mask_mode=mask_mode, mref=mref, scale=bn.scale, shift=bn.shift,
                       gout=gout, fin=fin)

    def _bwd_block(self, i: int):
        """Backward of block i. On entry its output gradient is already masked by the block's
        final ReLU and the tail BN statistics are accumulated: block i+1's last dgrad did both in
        its epilogue (BNBwdEpilogue, MASK_OUT). The last block does them with explicit passes."""
        b = self.blocks[i]
        N = self.N
        last = i == len(self.blocks) - 1
        x = self.p0 if i == 0 else self.blocks[i - 1].out
        nconv = len(b.convs)
        lc, lbn = b.convs[-1], b.bns[-1]
        cnt_last = N * lc.OH * lc.OW
        pend, gin = None, None  # BN-backward apply deferred into the next dgrad's prologue
        ds_fold = None  # ... and the downsample BN's, into the downsample dgrad
        fuse3 = self._fuse3(b, last)  # conv3's BN-backward apply + dgrad + wgrad in one kernel
        if last:
            # g = dlast * (out > 0) -> self.g_last ; tail BN reductions (and ds BN) from dlast
            K.bn_bwd_reduce(self.dlast, b.ys[-1], lbn.mean, lbn.invstd, lbn.bstats, mask_mode=K.MASK_OUT, mref=b.out)
            if b.ds_conv is not None:
                K.bn_bwd_reduce(self.dlast, b.yd, b.ds_bn.mean, b.ds_bn.invstd, b.ds_bn.bstats,
                                mask_mode=K.MASK_OUT, mref=b.out)
            fin = lbn.fin_b if self._cin(lbn, cnt_last) else None
            if fin is None:
                self._coeff(lbn, cnt_last)
            K.bn_bwd_apply(self.dlast, b.ys[-1], lbn.coeff, b.dys[-1], mask_mode=K.MASK_OUT, mref=b.out,
                           gout=self.g_last, fin=fin)
            g = self.g_last
        else:
            g = self.blocks[i + 1].dx
        # backward finalizes still to run for the tail BNs (else finished by block i+1's conv1 dgrad
        # epilogue): run standalone before a consumer that reads the coefficients from memory, or
        # handed to the apply pass that consumes them (coeff_in)
        todo = {} if last else ({id(lbn): (lbn, cnt_last)} if not self._fused_fin(lbn) else {})

        def ready(bn):  # the coefficients are in memory before the next launch
            if id(bn) in todo:
                self._coeff(*todo.pop(id(bn)))

        def fin_of(bn):  # the apply pass finalizes them itself (or they are ready)
            if id(bn) in todo and self._cin(*todo[id(bn)]):
                todo.pop(id(bn))
                return bn.fin_b
            ready(bn)
            return None

        if b.ds_conv is not None:
            dc, dbn = b.ds_conv, b.ds_bn
            if last or not self._fused_fin(dbn):
                todo[id(dbn)] = (dbn, N * dc.OH * dc.OW)
            if last:
                K.bn_bwd_apply(g, b.yd, dbn.coeff, b.dyd, mask_mode=K.MASK_NONE, fin=fin_of(dbn))
            elif (fuse3 or self._fold(lc)) and self._fold(dc, dense=True):
                # both tail BN applies folded into the dgrads of conv3 and of the downsample conv
                ready(lbn)
                ready(dbn)
                pend = dict(bwd_y=b.ys[-1], bwd_coeff=lbn.coeff, dy_out=b.dys[-1])
                gin = g
                ds_fold = dict(bwd_y=b.yd, bwd_coeff=dbn.coeff, dy_out=b.dyd)
            elif fuse3:  # conv3's inside the fused kernel, the downsample BN's as its own pass
                K.bn_bwd_apply(g, b.yd, dbn.coeff, b.dyd, mask_mode=K.MASK_NONE, fin=fin_of(dbn))
                ready(lbn)
                pend = dict(bwd_y=b.ys[-1], bwd_coeff=lbn.coeff, dy_out=b.dys[-1])
                gin = g
            else:  # both tail BNs from one read of the block-output gradient
                f1, f2 = fin_of(lbn), fin_of(dbn)
                K.bn_bwd_apply2(g, b.ys[-1], lbn.coeff, b.dys[-1], b.yd, dbn.coeff, b.dyd, fin1=f1, fin2=f2)
        elif not last:
            if fuse3 or self._fold(lc):  # folded into conv3's dgrad prologue (it stores dys[-1] for the wgrad)
                ready(lbn)
                pend = dict(bwd_y=b.ys[-1], bwd_coeff=lbn.coeff, dy_out=b.dys[-1])
                gin = g
            else:
                K.bn_bwd_apply(g, b.ys[-1], lbn.coeff, b.dys[-1], mask_mode=K.MASK_NONE, fin=fin_of(lbn))
        assert not todo, "a tail BN's backward finalize was left pending"
        # (the downsample conv's data gradient on a branch / the side stream beside the inner convs'
        # measured neutral or slower in round 5 and was removed: profiles/r5_side_defer/)
        # inner convs, last to second: dgrad epilogue masks with the previous BN's ReLU and
        # accumulates that BN's backward statistics
        for j in range(nconv - 1, 0, -1):
            cv, pbn, pc = b.convs[j], b.bns[j - 1], b.convs[j - 1]
            # dgrad first: its epilogue also stores the BN output acts[j-1] = this conv's input,
            # which the (side-stream) weight gradient then reads without a BN prologue
            act = b.acts[j - 1]
            kw, src = (pend, gin) if pend else ({}, b.dys[j])
            pend = None
            if fuse3 and j == nconv - 1:
                # one pass: dy3 = BN3-bwd apply(g, y3) -> da2 (+ BN2 moments) and dW3 = dy3^T relu(bn2(y2))
                K.conv_dwfused(src, kw["bwd_y"], kw["bwd_coeff"], cv.wt16, b.ys[j - 1], pbn.scale, pbn.shift,
                               pbn.mean, pbn.invstd, pbn.bstats, b.das[j - 1], cv.grad, self.ws_dw,
                               cus=self.dwf_cus if self.overlap_wgrad else 0)
                act, kw = None, None
            pre = act is None and kw == {}  # wgrad re-applies BN+ReLU to its staged input tiles (BN prologue)
            if pre:
                self._wgrad(b.dys[j], b.ys[j - 1], cv.grad, self.ws, R=cv.R, S=cv.S, stride=cv.stride, pad=cv.pad,
                            in_scale=pbn.scale, in_shift=pbn.shift, relu_in=True)
            if kw is not None:
                # (the forward materialised acts[j-1] already when b.mat[j-1]: no write-back)
                K.conv_dgrad(src, cv.wt16, b.das[j - 1], R=cv.R, S=cv.S, stride=cv.stride, pad=cv.pad,
                             epilogue=K.BNBwdEpilogue(K.MASK_Y, b.ys[j - 1], pbn.mean, pbn.invstd, pbn.bstats,
                                                      scale=pbn.scale, shift=pbn.shift,
                                                      act_out=None if b.mat[j - 1] else act,
                                                      fin1=pbn.fin_b if self._fused_fin(pbn) else None), **kw)
            if act is not None:
                self._wgrad(b.dys[j], act, cv.grad, self.ws, R=cv.R, S=cv.S, stride=cv.stride, pad=cv.pad)
            elif kw and not pre:
                self._wgrad(b.dys[j], b.ys[j - 1], cv.grad, self.ws, R=cv.R, S=cv.S, stride=cv.stride, pad=cv.pad,
                            in_scale=pbn.scale, in_shift=pbn.shift, relu_in=True)
            pcount = N * pc.OH * pc.OW
            fold = self._fold(pc)
            fin = None
            if kw is None or not self._fused_fin(pbn):  # (else finished by the dgrad epilogue above)
                if not fold and self._cin(pbn, pcount):
                    fin = pbn.fin_b  # finalized by the apply pass below
                else:
                    self._coeff(pbn, pcount)
            if fold:  # the next dgrad (conv j-1) applies it while staging
                pend = dict(bwd_y=b.ys[j - 1], bwd_coeff=pbn.coeff, dy_out=b.dys[j - 1])
                gin = b.das[j - 1]
            else:
                K.bn_bwd_apply(b.das[j - 1], b.ys[j - 1], pbn.coeff, b.dys[j - 1], mask_mode=K.MASK_NONE, fin=fin)
        # first conv: wgrad (after the dgrad when that stores dys[0]), then the block-input gradient
        # = dgrad(conv1) + shortcut gradient
        c0 = b.convs[0]
        kw0, src0 = (pend, gin) if pend else ({}, b.dys[0])
        if not kw0:
            self._wgrad(b.dys[0], x, c0.grad, self.ws, R=c0.R, S=c0.S, stride=c0.stride, pad=c0.pad)
        if b.ds_conv is not None:
            dc = b.ds_conv
            if ds_fold is None:
                self._wgrad(b.dyd, x, dc.grad, self.ws, R=dc.R, S=dc.S, stride=dc.stride, pad=dc.pad)
                # 1x1 strided downsample: its dgrad is a dense GEMM onto the stride-subsampled pixels
                K.conv_dgrad(b.dyd, dc.wt16, b.dsbuf, R=1, S=1, stride=1, pad=0)
            else:  # the dgrad computes (and stores) dyd from g; the wgrad follows it
                K.conv_dgrad(g, dc.wt16, b.dsbuf, R=1, S=1, stride=1, pad=0, **ds_fold)
                self._wgrad(b.dyd, x, dc.grad, self.ws, R=dc.R, S=dc.S, stride=dc.stride, pad=dc.pad)
            addsrc, sub = b.dsbuf, dc.stride
        else:
            addsrc, sub = g, 1
        epi = None
        if i > 0:
            pb = self.blocks[i - 1]
            epi = K.BNBwdEpilogue(K.MASK_OUT, pb.ys[-1], pb.bns[-1].mean, pb.bns[-1].invstd, pb.bns[-1].bstats,
                                  mbits=pb.obits,
                                  ybn2=pb.yd if pb.ds_conv is not None else None,
                                  mean2=pb.ds_bn.mean if pb.ds_conv is not None else None,
                                  inv2=pb.ds_bn.invstd if pb.ds_conv is not None else None,
                                  stats2=pb.ds_bn.bstats if pb.ds_conv is not None else None,
                                  fin1=pb.bns[-1].fin_b if self._fused_fin(pb.bns[-1]) else None,
                                  fin2=(pb.ds_bn.fin_b if pb.ds_conv is not None and self._fused_fin(pb.ds_bn)
                                        else None))
        K.conv_dgrad(src0, c0.wt16, b.dx, R=c0.R, S=c0.S, stride=c0.stride, pad=c0.pad,
                     addsrc=addsrc, add_sub=sub, epilogue=epi, **kw0)
        if kw0:
            self._wgrad(b.dys[0], x, c0.grad, self.ws, R=c0.R, S=c0.S, stride=c0.stride, pad=c0.pad)

    def fwd_conv_flops(self) -> float:
        """FLOPs of the forward convolutions of one step (sizes the wgrad side-stream decision)."""
        return sum(2.0 * self.N * cv.OH * cv.OW * cv.OC * cv.R * cv.S * cv.IC for cv in self.convs)

    def _materialize(self, cv: ConvL) -> bool:
        """Does conv ``cv`` (a block-internal 3x3) take a
        materialised BN output on the eight-wave kernel?"""
        if not (self.fast_mat and self.dev.type == "cuda" and cv.stride == 1
                and cv.R == 3):
            return False
        t = K.pick_tile(self.N * cv.OH * cv.OW, cv.OC, "fwd0", cv.IC, cv.R, cv.stride)
        return len(t) > 2 and t[2] in (4, 5)

    def _fuse3(self, b: BlockL, last: bool) -> bool:
        """Run block b's conv3 backward through K.conv_dwfused (the 64 -> 256 conv3 of the 56x56
        stage: its weight-gradient accumulators fit a workgroup's registers)."""
        if not self.fuse_dw or last or b.kind != "bottleneck":
            return False
        c3 = b.convs[-1]
        return ((c3.R, c3.S, c3.stride, c3.pad) == (1, 1, 1, 0) and c3.OH >= self.cfg.fuse_dw_min_hw
                and K.dwfused_preferred(c3.IC, c3.OC, self.N * c3.OH * c3.OW))

    def _fold(self, cv, dense: bool = False) -> bool:
        """Fold the BN-backward apply of cv's output BN into cv's dgrad (1x1 stride-1 convs;
        ``dense``: the strided 1x1 downsample, whose dgrad runs as a dense 1x1 stride-1 GEMM)."""
        stride = 1 if dense else cv.stride
        return (self.fuse_bwd_apply and not cv.stem and self.N * cv.OH * cv.OW * cv.OC >= self.fold_min
                and (cv.IC <= self.fold_max_ratio * cv.OC or cv.OH >= self.fold_ratio_min_hw)
                and K.tail_supported(cv.OC, cv.R, cv.S, stride, cv.pad))

    def _bwd_stem(self):
        st, sbn = self.stem, self.stem_bn
        dp = self.blocks[0].dx
        if K.pool_bn_bwd_supported(st.OC, self.pool_k, self.pool_s):
            # max-pool backward folded into the stem BN's reduce/apply passes (no pooled-grad tensor)
            pk = dict(K=self.pool_k, stride=self.pool_s, pad=self.pool_p)
            if self.pymax is not None:  # sum over windows of dpool * [y at argmax] == sum over pixels
                K.bn_bwd_reduce(dp, self.pymax, sbn.mean, sbn.invstd, sbn.bstats, mask_mode=K.MASK_Y,
                                scale=sbn.scale, shift=sbn.shift)
            else:
                K.pool_bn_bwd_reduce(dp, self.parg, self.y0, sbn.scale, sbn.shift, sbn.mean, sbn.invstd, sbn.bstats,
                                     **pk)
            K.bn_bwd_coeff(sbn.bstats, self.N * st.OH * st.OW, sbn.gamma, sbn.mean, sbn.invstd, sbn.coeff,
                           sbn.dgamma, sbn.dbeta)
            if self.fuse_stem_bwd and K.stem_bwd_supported(st.OC, self.pool_k, self.pool_s, st.R, st.S):
                # dy0 = BN-backward apply of the pool backward, straight into the weight-gradient tiles
                K.stem_bwd_fused(dp, self.parg, self.y0, sbn.scale, sbn.shift, sbn.coeff, self.x4, self.stem_grad_tmp,
                                 self.ws, R=st.R, S=st.S, conv_stride=st.stride, conv_pad=st.pad, **pk)
                g = self.grad[st.off:st.off + st.numel].view(st.OC, st.R, st.S, st.IC)
                g.copy_(self.stem_grad_tmp.view(st.OC, 8, 8, 4)[:, :st.R, :st.S, :st.IC])
                return
            K.pool_bn_bwd_apply(dp, self.parg, self.y0, sbn.scale, sbn.shift, sbn.coeff, self.dy0, **pk)
        else:
            K.maxpool_bwd(dp, self.parg, self.da0, K=self.pool_k, stride=self.pool_s, pad=self.pool_p)
            self._bn_bwd(sbn, self.da0, self.y0, self.dy0, self.N * st.OH * st.OW, K.MASK_Y)
        # small steps (stem_wg_main, see __init__): with the batched side stream the stem weight gradient
        # runs on the MAIN stream right here, next to the side stream's last batch (layer1's weight
        # gradients, forked at layer1's end) instead of queued behind it; its slabs live in ws_stem
        on_main = ((self.side_batch or self.side_block) and self.dev.type == "cuda" and self.overlap_wgrad
                   and self.stem_wg_main)

        def stem_wgrad():
            # reduced straight into the flat gradient's (OC, R, S, IC) slice when the stem tile kernel
            # runs (no padded temporary + strided copy)
            g = self.grad[st.off:st.off + st.numel]
            out = K.conv_wgrad(self.dy0, self.x4, self.stem_grad_tmp, self.ws_stem if on_main else self.ws, R=st.R,
                               S=st.S, stride=st.stride, pad=st.pad, stem=True, out_krsc=g)
            if out is not g:
                g.view(st.OC, st.R, st.S, st.IC).copy_(self.stem_grad_tmp.view(st.OC, 8, 8, 4)[:, :st.R, :st.S, :st.IC])
        if on_main:
            stem_wgrad()
        else:
            self._side(stem_wgrad)

    def backward(self):
        for _, fn in self._segments:
            fn()

    # parameter-name groups per backward segment (for bucket assembly)
    def segment_param_ranges(self) -> List[List[Tuple[str, int, int]]]:
        groups = []
        by_prefix = {"head": ["fc."], "layer4": ["layer4."], "layer3": ["layer3."], "layer2": ["layer2."],
                     "layer1": ["layer1."], "stem": ["conv1.", "bn1."]}
        for name, _ in self._segments:
            pre = by_prefix[name]
            groups.append([r for r in self.param_ranges if any(r[0].startswith(p) for p in pre)])
        return groups
