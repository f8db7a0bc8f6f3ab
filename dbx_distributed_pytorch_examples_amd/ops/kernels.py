"""Python front-ends of the HIP kernels (``csrc/*.hip``).

Every wrapper validates dtype / contiguity / shape on the host before launching (a mismatch
would otherwise be an out-of-bounds GPU access), launches on the current torch stream (so the
calls are captured by ``torch.cuda.graph``), and never synchronises. Layout conventions:

* activations: NHWC bf16, contiguous, ``[N, H, W, C]`` (C % 8 == 0; conv inputs C % 64 == 0,
  except the stem which takes the NHWC4 image);
* conv weights: KRSC bf16 ``[OC, R*S*IC]`` for forward, CRSK ``[IC, R*S*OC]`` for dgrad,
  the stem as ``[64, 8*8*4]`` (7x7x3 zero-padded to 8x8x4);
* BN statistics: fp64 ``[nshard, 2, C]`` slabs accumulated by conv epilogues (order-independent).
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import torch

from ..utils import debug as _debug
from . import reference as _ref
from ._ext import C, stream_ptr, use_native
from ..engine_config import EngineConfig

_E = EngineConfig.current  # kernel-selection switches (engine_config.py; DBX_ENGINE overrides)

FWD, DGRAD, STEM, FWD_PATCH, DGRAD_PATCH = 0, 1, 2, 3, 4
# addsrc, add_sub, epi, mbits, ybn, ybn2, bsc, bsh, mean1, inv1, mean2, inv2, bstats1, bstats2
_NO_EPI = (0, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0)
MASK_NONE, MASK_OUT, MASK_Y = 0, 1, 2


_POST_LAUNCH = None


def set_post_launch(cb, owner=None) -> None:
    """Run ``cb`` once, right after the next native kernel launch. ``cb=None`` cancels -- with
    ``owner`` given, only if the pending callback is ``owner`` (one program never cancels another's).
    The program's deferred side-stream batches use it to enter the captured graph after the main
    chain's next node."""
    global _POST_LAUNCH
    if cb is None and owner is not None and _POST_LAUNCH is not None and _POST_LAUNCH != owner:
        return
    _POST_LAUNCH = cb


def _dispatch(fn):
    """Run the HIP kernel for GPU tensors, the PyTorch reference (ops/reference.py) otherwise.
    With ``DBX_DEBUG=1`` every native launch is followed by a sync + output check (utils/debug.py)."""
    ref = getattr(_ref, fn.__name__)
    checked = _debug.checked_op(fn)

    def wrapper(*args, **kw):
        global _POST_LAUNCH
        t = args[0]
        if isinstance(t, torch.Tensor) and not use_native(t):
            return ref(*args, **kw)
        r = checked(*args, **kw) if _debug.enabled() else fn(*args, **kw)
        if _POST_LAUNCH is not None:
            cb, _POST_LAUNCH = _POST_LAUNCH, None
            cb()
        return r

    wrapper.__name__ = fn.__name__
    wrapper.__doc__ = fn.__doc__
    wrapper.__wrapped__ = fn
    return wrapper


NSHARD = _ref.NSHARD  # BN-statistics shards (spreads the epilogue atomics over NSHARD copies)


class BnFin:
    """In-launch BatchNorm finalize descriptor (csrc/abi.h BnFin, csrc/bn_fin.h): handed to the conv
    that accumulates a BN's statistics (``conv_fwd(fin=)`` for the forward statistics, ``BNBwdEpilogue
    (fin1=, fin2=)`` for the backward ones), it makes the producer's last tile of every 64-channel group
    compute what ``bn_finalize`` (mode 1) / ``bn_bwd_coeff`` (mode 2) would, bit for bit -- one launch
    and one graph node fewer per BN and direction. Producers that cannot (reference ops on the CPU,
    multi-launch strided dgrads, the stem) call :meth:`run` instead, so after the producer returns the
    finalize is done either way. The descriptor holds raw pointers: rebuild it if a tensor it names
    is reallocated."""

    FWD, BWD = 1, 2

    def __init__(self, mode, stats, count, *, gamma=None, beta=None, eps=1e-5, momentum=0.0, running_mean=None,
                 running_var=None, scale=None, shift=None, mean=None, invstd=None, coeff=None, dgamma=None,
                 dbeta=None, accumulate=False):
        C = (scale if mode == self.FWD else coeff).numel() // (1 if mode == self.FWD else 3)
        if C % 64:
            raise ValueError("BnFin needs a multiple of 64 channels")
        self.mode, self.stats, self.count, self.C = mode, stats, float(count), C
        self.gamma, self.beta, self.eps, self.momentum = gamma, beta, float(eps), float(momentum)
        self.running_mean, self.running_var, self.scale, self.shift = running_mean, running_var, scale, shift
        self.mean, self.invstd, self.coeff, self.dgamma, self.dbeta = mean, invstd, coeff, dgamma, dbeta
        self.accumulate = bool(accumulate)
        self.cnt = torch.zeros(C // 64, dtype=torch.int32, device=stats.device)
        self.desc = None
        if stats.is_cuda:
            import numpy as np
            ptrs = [self.cnt, stats, gamma, beta, running_mean, running_var, scale, shift, mean, invstd, coeff,
                    dgamma, dbeta]
            buf = np.zeros(136, dtype=np.uint8)
            buf[:104].view(np.uint64)[:] = [_p(t) for t in ptrs]
            buf[104:120].view(np.int32)[:] = [C, stats.numel() // (2 * C), mode, int(accumulate)]
            buf[120:136].view(np.float32)[:] = [count, eps, momentum, 0.0]
            self.desc = torch.from_numpy(buf).to(stats.device)

    def ptr(self) -> int:
        return self.desc.data_ptr() if self.desc is not None else 0

    def pair_ptr(self, other: "BnFin") -> int:
        """Device address of the two-descriptor array [self, other] (a forward tail prologue with a
        shortcut BN). Built on first use -- callers that capture graphs build it beforehand (the
        program's build_fins), so no copy kernel lands in a captured step."""
        if getattr(self, "_pair", None) is None or self._pair[0] is not other:
            self._pair = (other, torch.cat([self.desc, other.desc]))
        return self._pair[1].data_ptr()

    def run(self) -> None:
        """The standalone finalize launch (what the fused path replaces)."""
        if self.mode == self.FWD:
            bn_finalize(self.stats, self.count, self.gamma, self.beta, self.eps, self.momentum, self.running_mean,
                        self.running_var, self.scale, self.shift, self.mean, self.invstd)
        else:
            bn_bwd_coeff(self.stats, self.count, self.gamma, self.mean, self.invstd, self.coeff, self.dgamma,
                         self.dbeta, accumulate=self.accumulate)


def new_stats(C: int, device=None, nshard: Optional[int] = None) -> torch.Tensor:
    """Zeroed BN-statistics slab ``[nshard, 2, C]`` (flat, fp64: the epilogue atomics add fp32
    partials exactly, so statistics do not depend on tile completion order). ``nshard`` (default
    NSHARD, at most 32): the copies the producer's atomics are spread over; every kernel reads the
    count off the slab's size, so each BN may have its own."""
    return torch.zeros((nshard or NSHARD) * 2 * C, device=device, dtype=torch.float64)


def _p(t: Optional[torch.Tensor]) -> int:
    return 0 if t is None else t.data_ptr()


def _nsh(stats, C: int) -> int:
    """Shard count of a BN-statistics slab ``[nshard, 2, C]`` (fp64), from its size; NSHARD when absent."""
    if stats is None:
        return NSHARD
    n = stats.numel() // (2 * C)
    if n < 1 or n > 32 or n * 2 * C != stats.numel():
        raise ValueError(f"statistics slab of {stats.numel()} elements is not [nshard <= 32, 2, {C}]")
    return n


def _chk_stats(t: torch.Tensor, name: str, C: int) -> int:
    _chk(t, torch.float64, name)
    return _nsh(t, C)


def _chk(t: torch.Tensor, dtype, name: str, numel: Optional[int] = None):
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")
    if not t.is_cuda:
        raise ValueError(f"{name}: must be a GPU tensor")
    if numel is not None and t.numel() != numel:
        raise ValueError(f"{name}: expected {numel} elements, got {t.numel()} (shape {tuple(t.shape)})")
    if t.numel() >= 2 ** 31 - 256:
        # the conv gathers use 32-bit element offsets; split the batch above 2^31 elements
        raise ValueError(f"{name}: {t.numel()} elements exceed the kernels' 32-bit offset range")


def conv_out_hw(h: int, w: int, r: int, s: int, stride: int, pad: int) -> Tuple[int, int]:
    return (h + 2 * pad - r) // stride + 1, (w + 2 * pad - s) // stride + 1


_TUNE = None


def _tune_table():
    global _TUNE
    if _TUNE is None:
        import json
        import os
        p = _E().tune_table or os.path.join(os.path.dirname(os.path.abspath(__file__)), "tune_table.json")
        _TUNE = {}
        modes = _E().tune_modes.split(",")  # e.g. "none", "fwd,dgrad2"
        if os.path.exists(p):
            with open(p) as f:
                _TUNE = {k: tuple(v) for k, v in json.load(f).items() if "all" in modes or k.split(":")[0] in modes}
    return _TUNE


def tune_key(mode: str, M: int, OC: int, K_in: int, R: int, stride: int) -> str:
    return f"{mode}:M{M}:N{OC}:K{K_in}:R{R}:s{stride}"


def pick_tile(M: int, OC: int, mode: str = "fwd", K_in: int = 0, R: int = 0, stride: int = 1,
              use_table: bool = True) -> Tuple[int, int]:
    """Measured winner from ops/tune_table.json (tools/tune_conv.py) if present, else the
    heuristic: biggest tile that still puts >= ~2 workgroups on each of the 256 CUs."""
    if use_table:
        t = _tune_table().get(tune_key(mode, M, OC, K_in, R, stride))
        if t is None and (mode in ("fwdt", "fwd0") or mode.endswith("b")):  # variants: the base entry
            t = _tune_table().get(tune_key("fwd" if mode in ("fwdt", "fwd0") else mode[:-1], M, OC, K_in, R, stride))
            if t is not None and len(t) > 2 and t[2] in (4, 5) and mode != "fwd0":
                t = None  # an eight-wave (plain operand) entry does not serve the prologue variants
        if t is not None and len(t) > 2 and t[2] in (4, 5) and not _fast_enabled():
            t = None  # fast=0: no eight-wave kernel (A/B runs)
        if t is not None and OC % t[1] == 0:
            return t  # (bm, bn) or (bm, bn, dma): a measured operand path (tools/tune_conv.py)
    if OC % 128 == 0 and ((M + 127) // 128) * (OC // 128) >= 512:
        return 128, 128
    if ((M + 127) // 128) * (OC // 64) >= 384:
        return 128, 64
    return 64, 64




def _fast_enabled() -> bool:
    """``fast`` (default on): use the eight-wave kernel entries of the tune table (csrc/conv_fast.hip)."""
    return _E().fast


def _tile_dma(t) -> Tuple[int, int, int]:
    """(bm, bn[, dma]) -> (bm, bn, dma). ``dma`` is the conv operand path (conv_igemm_kernel.h):
    0 register-staged, 1 weights by LDS-DMA (prologue convs), 2 / 3 both operands by LDS-DMA
    through a 2- / 3-slot ring of 64-channel stages, 6 through a 4-slot ring of 32-channel stages
    (4 / 5: the eight-wave kernel; 7 was a row-tile kernel of the 1x1 BN-prologue forwards, measured
    slower in round 4 and removed in round 6). The engine's ``conv_dma`` overrides every
    choice (A/B runs)."""
    forced = _E().conv_dma
    if forced >= 0:
        return int(t[0]), int(t[1]), forced
    return int(t[0]), int(t[1]), int(t[2]) if len(t) > 2 else 0




def patch3_supported(IC: int, OC: int, R: int, S: int, stride: int, pad: int, H: int, W: int) -> bool:
    """Geometry of the weights-stationary 3x3 patch kernel (csrc/conv_patch3.hip)."""
    return (R == 3 and S == 3 and stride == 1 and pad == 1 and IC == 64 and OC == 64 and W == 56
            and H % 8 == 0)


def _use_patch3(tile, mode: str) -> int:
    """0 = implicit GEMM, 1 = patch kernel with resident weights (one workgroup per CU), 2 = patch
    kernel with streamed weights (two workgroups per CU). tile "patch" / "patch_r" / "patch_s"
    forces one, an explicit (bm, bn[, dma]) the implicit GEMM; otherwise the engine's ``patch3`` ("all" default,
    "fwd", "dgrad" or "0") picks the convs and ``patch3_stream`` ("dgrad" default, "fwd", "all",
    "0") the ones on the streamed-weights variant."""
    use, stream = _E().patch3, _E().patch3_stream
    kind = 2 if stream in ("all", mode) else 1
    if isinstance(tile, str):
        return {"patch": kind, "patch_r": 1, "patch_s": 2}.get(tile, 0)
    if tile is not None:
        return 0
    return kind if (use == "all" or mode in use.split(",")) else 0


# --------------------------------------------------------------------------------------
# convolutions
# --------------------------------------------------------------------------------------
@_dispatch
def conv_fwd(x, w16, out, *, R, S, stride, pad, stats=None, in_scale=None, in_shift=None,
             relu_in=True, tile=None, tail_res=None, tail_res_scale=None, tail_res_shift=None, tail_out=None,
             tail_bits=None, fin: "BnFin" = None, _split=True, _fin=(0, 1), fin_in: "BnFin" = None,
             fin_in_res: "BnFin" = None):
    """Y = conv(act(X), W); act = relu(X*in_scale + in_shift) with a BN prologue. "Tail" mode
    (``tail_res`` given; 1x1 stride-1 convs): act = relu(X*in_scale + in_shift + r), r = tail_res or
    tail_res*tail_res_scale + tail_res_shift -- the previous residual block's output computed on the
    fly -- and act / its 1-bit ReLU mask are stored to ``tail_out`` / ``tail_bits`` (bn_apply's
    outputs), so that pass and the re-read of the block output disappear. ``fin``: the BN finalize of
    ``stats`` (:class:`BnFin`), done by the launch's last tiles (or by a finalize launch after it).
    ``fin_in``: the forward finalize of the INPUT's BN (whose outputs are ``in_scale`` / ``in_shift``),
    done inside this launch's prologue where the kernel supports it, else by its standalone launch
    first -- either way it is complete when this returns."""
    N, IH, IW, IC = x.shape
    OH, OW = conv_out_hw(IH, IW, R, S, stride, pad)
    OC = w16.shape[0]
    _chk(x, torch.bfloat16, "x")
    _chk(w16, torch.bfloat16, "w16", OC * R * S * IC)
    _chk(out, torch.bfloat16, "out", N * OH * OW * OC)
    if IC % 64 or OC % 64:
        raise ValueError(f"conv_fwd needs IC,OC % 64 == 0 (got {IC},{OC})")
    if stats is not None:
        _chk_stats(stats, "stats", OC)
    if in_scale is not None:
        _chk(in_scale, torch.float32, "in_scale", IC)
        _chk(in_shift, torch.float32, "in_shift", IC)
    if tail_res is not None:
        if not tail_supported(IC, R, S, stride, pad) or in_scale is None or not relu_in:
            raise ValueError("tail prologue needs a 1x1 stride-1 conv, <= 1024 input channels and a BN prologue")
        _chk(tail_res, torch.bfloat16, "tail_res", x.numel())
        if tail_res_scale is not None:
            _chk(tail_res_scale, torch.float32, "tail_res_scale", IC)
            _chk(tail_res_shift, torch.float32, "tail_res_shift", IC)
        if tail_out is not None:
            _chk(tail_out, torch.bfloat16, "tail_out", x.numel())
        if tail_bits is not None:
            _chk(tail_bits, torch.uint8, "tail_bits", x.numel() // 8)
    mode = FWD
    kind = _use_patch3(tile, "fwd") if tail_res is None and patch3_supported(IC, OC, R, S, stride, pad, IH, IW) else 0
    if kind:
        mode, bm, bn, dma = FWD_PATCH, 0, 0, kind - 1
    else:
        if isinstance(tile, str):
            raise ValueError("tile='patch' needs a 64->64 3x3 stride-1 conv at width 56")
        plain = in_scale is None and tail_res is None
        bm, bn, dma = _tile_dma(tile or pick_tile(N * OH * OW, OC, "fwd0" if plain else
                                                  ("fwd" if tail_res is None else "fwdt"), IC, R, stride))
    if (tile is None and not kind and sweep_fwd_ok(N * OH * OW, IC, OC, R, S, stride, pad, in_scale is not None,
                                                    tail_res is None, relu_in)):
        bm, bn, dma = 128, 256, 8
    if dma in (4, 5) and (in_scale is not None or tail_res is not None):
        if tile is not None:
            raise ValueError("the eight-wave kernel (tile dma 4 / 5) takes plain operands (no BN prologue / tail)")
        bm, bn, dma = _tile_dma(pick_tile(N * OH * OW, OC, use_table=False))
    if dma == 5:  # eight-wave kernel over the whole batch (no split)
        dma = 4
    elif dma == 4 and _split:
        n1 = fast_split(N, OH * OW, OC, bn)
        kw = dict(R=R, S=S, stride=stride, pad=pad, stats=stats, fin=fin, _split=False)
        if n1 > 0:  # (the fast launch's tiles count toward the finalize the leftover launch completes)
            conv_fwd(x[:n1], w16, out[:n1], tile=(256, bn, 4), _fin=(0, int(n1 == N)), **kw)
        if n1 < N:  # the leftover images on small four-wave tiles (they fill the chip)
            conv_fwd(x[n1:], w16, out[n1:], tile=pick_tile((N - n1) * OH * OW, OC, use_table=False),
                     _fin=(-(-n1 * OH * OW // 256), 1), **kw)
        return out
    f1 = fin.ptr() if fin is not None and stats is not None else 0
    fi = 0
    if fin_in is not None or fin_in_res is not None:
        pair = tail_res is not None and tail_res_scale is not None
        fins = [f for f in (fin_in, fin_in_res if pair else None) if f is not None]
        if (mode == FWD and in_scale is not None and dma in (0, 1) and fin_in is not None
                and all(f.desc is not None for f in fins) and (not pair or fin_in_res is not None)):
            # the implicit-GEMM prologue finalizes it (csrc/bn_fin.h bn_fin_consume); a forward
            # tail with a shortcut BN takes both descriptors as one array
            fi = fin_in.ptr() if not pair else fin_in.pair_ptr(fin_in_res)
        else:
            for f in fins:
                f.run()
        if fin_in_res is not None and not pair:
            fin_in_res.run()
    r0, nr = fwd_taps(IH, OH, R, stride, pad)
    s0, ns = fwd_taps(IW, OW, S, stride, pad)
    if nr == 0 or ns == 0:
        raise ValueError("conv_fwd: no filter tap touches the input")
    sk = (conv_splitk(N * OH * OW, OC, bm, bn, dma, nr * ns * (IC // (32 if dma == 6 else 64)))
          if mode == FWD else (1, 0, 0, 0))
    C().conv_igemm(mode, bm, bn, x.data_ptr(), w16.data_ptr(), out.data_ptr(), _p(in_scale), _p(in_shift),
                   int(relu_in), _p(stats), _nsh(stats, OC), N, IH, IW, IC, OH, OW, OC, R, S, stride, pad, 0,
                   nr, ns, r0, s0, 1, 0, 0, 1, 0, 0, OH, OW, *_NO_EPI, 0, _p(tail_res), _p(tail_res_scale),
                   _p(tail_res_shift), _p(tail_out), _p(tail_bits), stream_ptr(), dma, f1, 0, _fin[0], _fin[1], fi,
                   *sk)
    if fin is not None and not f1 and _fin[1]:
        fin.run()
    return out


_SK_BUFS = {}   # stream -> [fp32 slab workspace, tile counters] of the split-K conv launches
_SK_KEEP = []   # every buffer ever handed out (a captured graph keeps using its pointers)


def sweep_fwd_ok(M: int, IC: int, OC: int, R: int, S: int, stride: int, pad: int, pro: bool, no_tail: bool,
                 relu_in: bool) -> bool:
    """Does the N-sweep kernel (csrc/conv_sweep.hip, tile code dma 8) take this forward? 1x1 stride-1
    BN-prologue (+ReLU) convs with K <= 256 input channels, a multiple of 256 output channels, and
    enough 128-row blocks to keep every CU on several of them (the engine's ``sweep_fwd``)."""
    cfg = _E()
    return (cfg.sweep_fwd and pro and no_tail and relu_in and (R, S, stride, pad) == (1, 1, 1, 0)
            and IC % 64 == 0 and IC <= 256 and OC % 256 == 0
            and -(-M // 128) >= cfg.sweep_min_tiles_per_cu * num_cus())


def sweep_dgrad_ok(M: int, K: int, Cc: int, R: int, S: int, stride: int, pad: int, fold: bool, add_sub: int,
                   epi_mode: int) -> bool:
    """Does the N-sweep kernel take this data gradient? The folded 1x1 stride-1 dgrads (BN-backward apply
    in the operand staging) of <= 256 channels onto a multiple of 256, with an addend at full resolution
    and no or the MASK_OUT epilogue (the engine's ``sweep_dgrad``)."""
    cfg = _E()
    return (cfg.sweep_dgrad and fold and (R, S, stride, pad) == (1, 1, 1, 0) and add_sub == 1
            and epi_mode in (0, MASK_OUT) and K % 64 == 0 and K <= 256 and Cc % 256 == 0
            and -(-M // 128) >= cfg.sweep_min_tiles_per_cu * num_cus())


def conv_splitk(M: int, OC: int, bm: int, bn: int, dma: int, KB: int) -> Tuple[int, int, int, int]:
    """Split-K plan of one implicit-GEMM launch: (ksplit, kper, slab ptr, counter ptr); (1, 0, 0, 0) =
    no split. Few-tile launches (fewer than the engine's ``splitk_wgs`` tiles: the 4x4 / 2x2 maps of
    the TinyImageNet step) walk their K blocks as one chain of HBM / L2 latencies per workgroup;
    slices of >= ``splitk_min_kb`` blocks run those chains side by side and the tile's last slice sums
    the fp32 partials in slice order (csrc/conv_igemm_kernel.h splitk_combine: bit-identical whichever
    slice finishes last). The slab / counter buffers are per stream (launches on one stream are
    ordered; the side stream's downsample forward runs beside the main stream's convs). The plan never
    depends on the buffers: a graph capture on a fresh stream allocates its own (from the graph's pool,
    kept alive here), so captured and eager steps split alike and agree bit for bit."""
    cfg = _E()
    ntile = -(-M // bm) * (OC // bn)
    if cfg.splitk_wgs <= 0 or dma not in (0, 1) or ntile >= cfg.splitk_wgs:
        return 1, 0, 0, 0
    s = min(cfg.splitk_wgs // ntile, KB // max(1, cfg.splitk_min_kb))
    if s < 2:
        return 1, 0, 0, 0
    kper = -(-KB // s)
    s = -(-KB // kper)  # every slice non-empty
    if s < 2:
        return 1, 0, 0, 0
    need_ws, need_cnt = s * ntile * bm * bn, ntile
    key = stream_ptr()
    bufs = _SK_BUFS.get(key)
    if bufs is None or bufs[0].numel() < need_ws or bufs[1].numel() < need_cnt:
        dev = torch.device("cuda", torch.cuda.current_device())
        nws = max(need_ws, bufs[0].numel() if bufs else 0)
        ncnt = max(need_cnt, bufs[1].numel() if bufs else 0, 4096)
        bufs = [torch.empty(nws, device=dev, dtype=torch.float32), torch.zeros(ncnt, device=dev, dtype=torch.int32)]
        _SK_BUFS[key] = bufs
        _SK_KEEP.append(bufs)
    return s, kper, bufs[0].data_ptr(), bufs[1].data_ptr()


def fast_split(N: int, per_img: int, OC: int, bn: int) -> int:
    """Images handled by the eight-wave kernel (csrc/conv_fast.hip: one 256 x bn tile per CU, one
    workgroup per CU) when the rest of the batch goes to the four-wave kernel: the fast launch covers
    only FULL rounds of num_cus() tiles (a partial last round would leave most CUs idle for a whole
    tile time: 784 tiles on 256 CUs = 3.06 rounds = 4 tile times); the leftover images run as
    small tiles that fill the chip. Returns N (no split), 0 (no full round: don't use the fast kernel)
    or the split point."""
    P = num_cus()
    ntn = OC // bn
    ntile = -(-N * per_img // 256) * ntn
    if ntile % P == 0:
        return N
    full_m = (ntile // P) * P // ntn * 256
    return min(N, full_m // per_img)


def tail_supported(IC: int, R: int, S: int, stride: int, pad: int) -> bool:
    """Can a conv consume the previous block's output through the fused tail prologue?"""
    return R == 1 and S == 1 and stride == 1 and pad == 0 and IC <= 1024 and IC % 64 == 0




def _prune() -> bool:
    """``tap_prune`` (default on): conv launches skip the filter taps that only ever see padding."""
    return _E().tap_prune


def fwd_taps(IH: int, OH: int, R: int, stride: int, pad: int) -> Tuple[int, int]:
    """(r0, nr): the filter rows of a forward conv that touch the image for SOME output row, i.e.
    0 <= oh*stride - pad + r < IH for an oh in [0, OH). The K loop skips the rest: on small maps
    (ResNet-18 at 32x32: layer4 is 1x1, so a 3x3 conv is its centre tap) the other taps would only
    multiply zero padding -- 8 of 9 K blocks of work and weight traffic."""
    if not _prune():
        return 0, R
    lo = max(0, pad - (OH - 1) * stride)
    hi = min(R - 1, IH - 1 + pad)
    return (lo, hi - lo + 1) if hi >= lo else (0, 0)


def _live_taps(n_out: int, d0: int, n_in: int, nt: int) -> Tuple[int, int]:
    """Tap indices t in [0, nt) with 0 <= i + d0 - t < n_in for some i in [0, n_out) (the transposed
    gather of a dgrad phase): (first, count)."""
    if not _prune():
        return 0, nt
    lo = max(0, d0 - n_in + 1)
    hi = min(nt - 1, n_out - 1 + d0)
    return (lo, hi - lo + 1) if hi >= lo else (0, 0)


def dgrad_phases(H: int, W: int, R: int, S: int, stride: int, pad: int):
    """Parity decomposition of a strided dgrad into stride-1 sub-problems.

    Output pixel h receives tap r only where (h + pad - r) % stride == 0, so for each output
    phase (ph, pw) only taps r = r0 + stride*t contribute and the gather is dense:
    ih = i + (ph + pad - r0) // stride - t over the phase's sub-grid i (h = i*stride + ph).
    Taps whose gather never lands inside dY (small maps: only padding) are dropped from the range.
    Returns [(ph, pw, OHs, OWs, r0, nr, s0, ns, dh0, dw0)] (classes with no taps included, nr=0).
    """
    P = (H + 2 * pad - R) // stride + 1
    Q = (W + 2 * pad - S) // stride + 1
    out = []
    for ph in range(stride):
        for pw in range(stride):
            ohs = (H - ph + stride - 1) // stride
            ows = (W - pw + stride - 1) // stride
            r0 = (ph + pad) % stride
            s0 = (pw + pad) % stride
            nr = max(0, (R - r0 + stride - 1) // stride)
            ns = max(0, (S - s0 + stride - 1) // stride)
            dh0, dw0 = (ph + pad - r0) // stride, (pw + pad - s0) // stride
            tr, nr = _live_taps(ohs, dh0, P, nr)
            ts, ns = _live_taps(ows, dw0, Q, ns)
            out.append((ph, pw, ohs, ows, r0 + stride * tr, nr, s0 + stride * ts, ns, dh0 - tr, dw0 - ts))
    return out


class BNBwdEpilogue:
    """Fused BN-backward epilogue for a dgrad: the dgrad result X (plus any residual addend) is
    masked — by the 1-bit mask ``mbits`` (mode MASK_OUT: the ReLU after a residual add, bits written
    by ``bn_apply(..., mbits=)`` for the block output)
    or by ``ybn*scale+shift > 0`` (MASK_Y: the ReLU after this BN) — and written as g, while
    ``stats1 += [sum g, sum g*xhat(ybn)]`` (and ``stats2 += [sum g, sum g*xhat(ybn2)]`` for a second
    BN fed by the same gradient: the downsample branch). Replaces a separate reduction pass."""

    def __init__(self, mode, ybn, mean1, inv1, stats1, mbits=None, scale=None, shift=None,
                 ybn2=None, mean2=None, inv2=None, stats2=None, act_out=None, fin1=None, fin2=None):
        self.mode, self.ybn, self.mean1, self.inv1, self.stats1 = mode, ybn, mean1, inv1, stats1
        self.act_out = act_out  # MASK_Y only: also store relu(ybn*scale+shift) (the BN output)
        self.mbits, self.scale, self.shift = mbits, scale, shift
        self.ybn2, self.mean2, self.inv2, self.stats2 = ybn2, mean2, inv2, stats2
        # BnFin (mode BWD) of stats1 / stats2: the backward coefficients are final when the dgrad returns
        self.fin1, self.fin2 = fin1, fin2

    def run_fin(self):
        for f in (self.fin1, self.fin2):
            if f is not None:
                f.run()

    def batch_slice(self, n0: int, n1: int, N: int) -> "BNBwdEpilogue":
        """The same epilogue over images [n0, n1) of an N-image batch (per-pixel tensors sliced)."""
        def sl(t):
            return None if t is None else t.view(N, -1)[n0:n1]
        return BNBwdEpilogue(self.mode, sl(self.ybn), self.mean1, self.inv1, self.stats1, mbits=sl(self.mbits),
                             scale=self.scale, shift=self.shift, ybn2=sl(self.ybn2), mean2=self.mean2, inv2=self.inv2,
                             stats2=self.stats2, act_out=sl(self.act_out), fin1=self.fin1, fin2=self.fin2)

    def args(self):
        return (self.mode, _p(self.mbits), _p(self.ybn), _p(self.ybn2), _p(self.scale), _p(self.shift),
                _p(self.mean1), _p(self.inv1), _p(self.mean2), _p(self.inv2), _p(self.stats1), _p(self.stats2))


@_dispatch
def conv_dgrad(dy, wt16, dx, *, R, S, stride, pad, accumulate=False, tile=None, addsrc=None, add_sub=1,
               epilogue: "BNBwdEpilogue" = None, bwd_y=None, bwd_coeff=None, dy_out=None, _split=True,
               _fin=(0, 1)):
    """dX = conv_transpose(dY, W): dy [N,P,Q,K], wt16 [C, R*S*K] (CRSK), dx [N,H,W,C].

    Stride > 1 runs one dense launch per output phase (``dgrad_phases``): no MFMA work on the
    (stride^2 - 1)/stride^2 taps that a masked gather would multiply by zero.
    ``accumulate``: dx += result (addsrc=None) or dx = result + addsrc (addsrc at 1/add_sub
    resolution, e.g. the dense dgrad of a strided 1x1 downsample); ``epilogue``: fused BN backward.
    ``bwd_y``/``bwd_coeff`` (1x1 stride-1 only): ``dy`` is the raw BN-output gradient g and the
    operand is the BN-backward apply k1*g + k2*bwd_y + k3 (coeff [3, K]) computed while staging;
    it is also stored to ``dy_out`` (for the weight gradient) -- bn_bwd_apply folded in.
    The epilogue's ``fin1`` / ``fin2`` (:class:`BnFin`) are done when this returns.
    """
    N, P, Q, K = dy.shape
    _, H, W, Cc = dx.shape
    _chk(dy, torch.bfloat16, "dy")
    _chk(wt16, torch.bfloat16, "wt16", Cc * R * S * K)
    _chk(dx, torch.bfloat16, "dx")
    if (H + 2 * pad - R) // stride + 1 != P or (W + 2 * pad - S) // stride + 1 != Q:
        raise ValueError("conv_dgrad: dy / dx shapes inconsistent with the conv geometry")
    if K % 64 or Cc % 64:
        raise ValueError("conv_dgrad needs channels % 64 == 0")
    if addsrc is not None:
        _chk(addsrc, torch.bfloat16, "addsrc", N * (H // add_sub) * (W // add_sub) * Cc)
        if H % add_sub or W % add_sub:
            raise ValueError("addsrc subsampling must divide the output size")
        accumulate = True
    epi = (0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0)
    nsh = NSHARD
    if epilogue is not None:
        e = epilogue
        _chk(e.ybn, torch.bfloat16, "ybn", dx.numel())
        nsh = _chk_stats(e.stats1, "stats1", Cc)
        if e.mode == MASK_OUT:
            _chk(e.mbits, torch.uint8, "mbits", dx.numel() // 8)
        if e.ybn2 is not None:
            _chk(e.ybn2, torch.bfloat16, "ybn2", dx.numel())
            if _chk_stats(e.stats2, "stats2", Cc) != nsh:
                raise ValueError("stats1 / stats2 must have the same shard count")
        if e.act_out is not None:
            if e.mode != MASK_Y:
                raise ValueError("act_out needs the MASK_Y epilogue")
            _chk(e.act_out, torch.bfloat16, "act_out", dx.numel())
        epi = e.args()
        act_ptr = _p(e.act_out)
        fins = (e.fin1.ptr() if e.fin1 is not None else 0, e.fin2.ptr() if e.fin2 is not None and e.stats2 is not None else 0)
        if fins[1] and not fins[0]:
            fins = (0, 0)
    else:
        act_ptr = 0
        fins = (0, 0)
    bwd = (0, 0, 0, 0, 0, 0)  # in_scale, in_shift, res, res_scale, res_shift, tail_out
    if bwd_y is not None:
        if not tail_supported(K, R, S, stride, pad):
            raise ValueError("BN-backward prologue needs a 1x1 stride-1 dgrad with <= 1024 channels")
        _chk(bwd_y, torch.bfloat16, "bwd_y", dy.numel())
        _chk(bwd_coeff, torch.float32, "bwd_coeff", 3 * K)
        if dy_out is not None:
            _chk(dy_out, torch.bfloat16, "dy_out", dy.numel())
        c0 = bwd_coeff.data_ptr()
        bwd = (c0, c0 + 8 * K, bwd_y.data_ptr(), c0 + 4 * K, 0, _p(dy_out))
    kind = (_use_patch3(tile, "dgrad") if not accumulate and bwd_y is None and (epilogue is None or epilogue.mode == MASK_Y)
            and patch3_supported(K, Cc, R, S, stride, pad, H, W) else 0)
    if kind:
        C().conv_igemm(DGRAD_PATCH, 0, 0, dy.data_ptr(), wt16.data_ptr(), dx.data_ptr(), 0, 0, 0, 0, nsh,
                       N, P, Q, K, H, W, Cc, R, S, stride, pad, 0, R, S, 0, 0, 1, 0, 0, 1, 0, 0, H, W,
                       0, 1, *epi, act_ptr, 0, 0, 0, 0, 0, stream_ptr(), kind - 1, *fins, 0, 1, 0, 1, 0, 0, 0)
        _fin_rest(epilogue, fins)
        return dx
    if isinstance(tile, str):
        raise ValueError("tile='patch' needs a 64->64 3x3 stride-1 dgrad at width 56 (no addend / fold)")
    if tile is None and sweep_dgrad_ok(N * H * W, K, Cc, R, S, stride, pad, bwd_y is not None, add_sub,
                                       epilogue.mode if epilogue is not None else 0):
        tile = (128, 256, 8)
    t_sel = tile
    if t_sel is None:
        t_sel = pick_tile(N * H * W, Cc, f"dgrad{epilogue.mode if epilogue else 0}" + ("b" if bwd_y is not None else ""),
                          K, R, stride)
    if t_sel is not None and _tile_dma(t_sel)[2] in (4, 5) and (bwd_y is not None or stride != 1 or add_sub != 1):
        if tile is not None:
            raise ValueError("the eight-wave kernel (tile dma 4 / 5) runs stride-1 dgrads without fold / subsampled addend")
        tile = t_sel = pick_tile(N * H * W, Cc, use_table=False)  # not eligible: the four-wave kernel
    if t_sel is not None and _tile_dma(t_sel)[2] == 5:
        tile = (256, _tile_dma(t_sel)[1], 4)  # eight-wave kernel over the whole batch (no split)
    elif t_sel is not None and _tile_dma(t_sel)[2] == 4 and _split:
        bn = _tile_dma(t_sel)[1]
        n1 = fast_split(N, H * W, Cc, bn)
        fins_of = ((0, int(n1 == N)), (-(-n1 * H * W // 256), 1))  # the leftover launch completes the count
        for (a0, a1, t), fi in zip(((0, n1, (256, bn, 4)), (n1, N, pick_tile((N - n1) * H * W, Cc, use_table=False))),
                                   fins_of):
            if a1 > a0:
                conv_dgrad(dy[a0:a1], wt16, dx[a0:a1], R=R, S=S, stride=stride, pad=pad, accumulate=accumulate,
                           tile=t, addsrc=None if addsrc is None else addsrc[a0:a1], add_sub=add_sub,
                           epilogue=None if epilogue is None else epilogue.batch_slice(a0, a1, N), _split=False,
                           _fin=fi)
        return dx
    phases = dgrad_phases(H, W, R, S, stride, pad)
    if not accumulate and any(ph[5] == 0 or ph[7] == 0 for ph in phases):
        if epilogue is not None:
            raise ValueError("fused BN epilogue needs every output pixel covered by one launch")
        dx.zero_()  # phases without taps receive no contribution
        accumulate = True
    if len(phases) > 1:  # several launches of differing tiles: finalize with its own launch
        fins = (0, 0)
    for (ph, pw, ohs, ows, r0, nr, s0, ns, dh0, dw0) in phases:
        if nr == 0 or ns == 0 or ohs == 0 or ows == 0:
            if epilogue is not None or addsrc is not None:
                raise ValueError("strided dgrad with empty phases cannot carry an epilogue / addend")
            continue
        bm, bn, dma = _tile_dma(tile or pick_tile(N * ohs * ows, Cc, f"dgrad{epilogue.mode if epilogue else 0}"
                                                  + ("b" if bwd_y is not None else ""), K, R, stride))
        sk = conv_splitk(N * ohs * ows, Cc, bm, bn, dma, nr * ns * (K // (32 if dma == 6 else 64)))
        if dma == 8:  # the N-sweep kernel takes its grid cap in the (unused) split-K slice field
            sk = (1, _E().sweep_dgrad_wgs, 0, 0)
        C().conv_igemm(DGRAD, bm, bn, dy.data_ptr(), wt16.data_ptr(), dx.data_ptr(), bwd[0], bwd[1], 0, 0, nsh,
                       N, P, Q, K, ohs, ows, Cc, R, S, stride, pad, int(accumulate),
                       nr, ns, r0, s0, stride, dh0, dw0, stride, ph, pw, H, W,
                       _p(addsrc), add_sub, *epi, act_ptr, bwd[2], bwd[3], bwd[4], bwd[5], 0, stream_ptr(), dma,
                       *fins, _fin[0], _fin[1], 0, *sk)
    if _fin[1]:
        _fin_rest(epilogue, fins)
    return dx


def _fin_rest(epilogue, fins) -> None:
    """Run the standalone finalize of every BnFin of ``epilogue`` the launch did not take."""
    if epilogue is None:
        return
    if epilogue.fin1 is not None and not fins[0]:
        epilogue.fin1.run()
    if epilogue.fin2 is not None and not fins[1]:
        epilogue.fin2.run()


def stem_patch_supported(IH: int, IW: int, OC: int, R: int, S: int, stride: int, pad: int) -> bool:
    """Geometry of the stem patch kernel (csrc/conv_patch3.hip): the ResNet 7x7/2 stem at 224."""
    OH, OW = conv_out_hw(IH, IW, R, S, stride, pad)
    return (R, S, stride, pad, IW, OC) == (7, 7, 2, 3, 224, 64) and OH % 4 == 0


@_dispatch
def conv_stem_fwd(x4, w16s, out, *, R=7, S=7, stride=2, pad=3, stats=None, patch=None):
    """Stem conv on the NHWC4 image: w16s [OC, 256] = (8 rows x 8 pixels x 4 channels).
    ``patch``: the patch kernel (224-wide images) -- None = the engine's ``stem_patch`` (default on)."""
    N, IH, IW, C4 = x4.shape
    if C4 != 4:
        raise ValueError("stem expects NHWC4 input")
    OH, OW = conv_out_hw(IH, IW, R, S, stride, pad)
    OC = w16s.shape[0]
    _chk(x4, torch.bfloat16, "x4")
    _chk(w16s, torch.bfloat16, "w16s", OC * 256)
    _chk(out, torch.bfloat16, "out", N * OH * OW * OC)
    if stats is not None:
        _chk_stats(stats, "stats", OC)
    if R > 8 or S > 8:
        raise ValueError("stem kernel supports R,S <= 8")
    if patch is None:
        patch = _E().stem_patch
    bm = 0 if patch and stem_patch_supported(IH, IW, OC, R, S, stride, pad) else 128  # bm 0: patch kernel
    C().conv_igemm(STEM, bm, 64, x4.data_ptr(), w16s.data_ptr(), out.data_ptr(), 0, 0, 0, _p(stats), _nsh(stats, OC),
                   N, IH, IW, 4, OH, OW, OC, R, S, stride, pad, 0, R, S, 0, 0, 1, 0, 0, 1, 0, 0, OH, OW,
                   *_NO_EPI, 0, 0, 0, 0, 0, 0, stream_ptr(), 0, 0, 0, 0, 1, 0, 1, 0, 0, 0)
    return out




def _stem_wgrad_tile() -> bool:
    """``stem_wgrad``: "tile" (default) = the 64 x 256-tile stem weight gradient (csrc/stem_bwd.hip),
    "generic" = the wgrad kernel's STEM mode (two 128-column tiles; A/B switch)."""
    return _E().stem_wgrad == "tile"


def wgrad_splits(M: int, OC: int, KTOT: int, bm: int, bn: int, max_ws_elems: int,
                 rounds: Optional[float] = None, cus: Optional[int] = None) -> Tuple[int, int]:
    """Split the pixel reduction so that ``rounds`` rounds of workgroups stream over the CUs (>= 8
    K-blocks each); the workspace holds nsplit slabs + up to 64 level-1 partial slabs of the
    reduction. ``rounds``: the tune table's per-shape value, else the engine's ``wgrad_rounds`` (2); 0 = no split
    (one workgroup per tile over all M rows, the gradient written directly)."""
    r = _E().wgrad_rounds if rounds is None else float(rounds)
    if r <= 0:
        return 1, max(64, (M + 63) // 64 * 64)
    tiles = (OC // bm) * (KTOT // bn)
    # r rounds of workgroups over the CUs (8-wave (256-wide) tiles run one per CU, 4-wave two):
    # fewer rounds = longer workgroups and proportionally smaller fp32 partial slabs
    ncu = num_cus() if cus is None else cus  # (cus: a side-stream launch sized to leave CUs free)
    target = max(1, int(r * (ncu if max(bm, bn) >= 256 else 2 * ncu)) // tiles)
    ms = max(512, ((M + target - 1) // target + 63) // 64 * 64)
    nsplit = (M + ms - 1) // ms
    while (nsplit + min(64, nsplit)) * OC * KTOT > max_ws_elems and nsplit > 1:
        ms *= 2
        nsplit = (M + ms - 1) // ms
    return nsplit, ms




def wgrad_fuse_max() -> int:
    """Largest per-tile slab volume (nsplit x BM x BN x 4 bytes) reduced inside the weight-gradient
    launch by the tile's last block (``wgrad_fuse_max`` bytes; 0 = always a separate reduce)."""
    return _E().wgrad_fuse_max


def wgrad_tiles_max(OC: int, KTOT: int) -> int:
    """Upper bound on the weight-gradient tile count of an OC x KTOT gradient (64 x 64 tiles): the
    size of its in-launch reduction counter slice."""
    return (OC // 64) * (KTOT // 64)


class ReduceBatch:
    """Deferred split-K reductions of a batch of weight gradients (the program's side-stream batch
    of one backward segment): each gradient's slabs go to its own region of ``arena`` and
    :meth:`flush` finishes them all with two launches (csrc/conv_igemm.hip dbx_wgrad_reduce_multi_run:
    level 1 of the two-level reductions, then every final sum) instead of one or two per gradient --
    bit-identical to ``wgrad_reduce`` in eager execution. A gradient whose slabs do not fit the
    arena's remainder is reduced at once (``need`` records the size the arena should grow to).

    The program uses it for its smallest steps (engine/program.py ``_flush_side``, ``defer_reduce``)."""

    def __init__(self, arena: torch.Tensor, start: int = 0, max_slab_bytes: Optional[int] = None):
        self.arena, self.off, self.need, self.jobs = arena, start, start, []
        # gradients whose slabs are larger are reduced at once (their slabs are still in L2 then)
        self.max_slab_bytes = max_slab_bytes

    def alloc(self, n: int):
        self.need += n
        if self.off + n > self.arena.numel():
            return None
        r = self.arena[self.off:self.off + n]
        self.off += n
        return r

    def add(self, ws, dw, n, nsplit, scale, accumulate):
        self.jobs.append((ws.data_ptr(), dw.data_ptr(), int(n), int(nsplit), float(scale), int(accumulate)))

    # device job tables by job list: built in eager steps, reused (never freed: captured graphs
    # read them) when the same batch is captured
    _tables: dict = {}

    def flush(self):
        jobs, self.jobs = tuple(self.jobs), []
        if not jobs:
            return
        ent = ReduceBatch._tables.get(jobs)
        if ent is None:
            if torch.cuda.is_current_stream_capturing() or len(ReduceBatch._tables) >= 4096:
                # no table for this batch (it was never run eagerly): reduce gradient by gradient
                for ws, dw, n, nsplit, scale, acc in jobs:
                    C().wgrad_reduce(ws, dw, n, nsplit, scale, acc, stream_ptr())
                return
            host = torch.empty(len(jobs) * C().wgrad_reduce_job_bytes(), dtype=torch.uint8)
            cols = [list(c) for c in zip(*jobs)]
            ga, gb = C().wgrad_reduce_multi_plan(*cols, host.data_ptr())
            dev = torch.empty_like(host, device=torch.device("cuda", torch.cuda.current_device()))
            dev.copy_(host)  # ordered on the current stream, before the launches below
            ent = ReduceBatch._tables[jobs] = (dev, ga, gb)
        dev, ga, gb = ent
        C().wgrad_reduce_multi_run(dev.data_ptr(), len(jobs), ga, gb, stream_ptr())


@_dispatch
def conv_wgrad(dy, x, dw, ws, *, R, S, stride, pad, in_scale=None, in_shift=None, relu_in=True,
               scale=1.0, accumulate=False, stem=False, tile=None, lds_pad=0, dma=-1, cnt=None, out_krsc=None,
               rounds=None, defer: "ReduceBatch" = None, cu_reserve: int = 0):
    """dW[OC, R*S*IC] (fp32, KRSC) = sum_pixels dY^T * im2col(X) ; ws = fp32 workspace.
    ``dma``: operand path of the prologue-free kernels -- LDS-DMA ring depth 2 / 3, 0 = register
    staged, -1 = the tune table's choice, else 3 for 256-wide tiles / 2.
    ``cnt``: zeroed int32 tile counters (>= wgrad_tiles_max(OC, KTOT), owned by this call site):
    when given and the split slabs of a tile are small (wgrad_fuse_max), the split-K reduction runs
    inside the launch (the last block of each tile sums its slabs, bit-identical to wgrad_reduce)
    and no separate reduce kernel is launched; one split writes dW directly. ``out_krsc`` (stem
    only): the reduction writes the real taps straight into this (OC, R, S, IC) gradient instead of
    the padded (OC, 8, 8, 4) ``dw``."""
    N, OH, OW, OC = dy.shape
    _, IH, IW, IC = x.shape
    KTOT = 256 if stem else R * S * IC
    _chk(dy, torch.bfloat16, "dy")
    _chk(x, torch.bfloat16, "x")
    _chk(dw, torch.float32, "dw", OC * KTOT)
    _chk(ws, torch.float32, "ws")
    if conv_out_hw(IH, IW, R, S, stride, pad) != (OH, OW):
        raise ValueError("conv_wgrad: shapes inconsistent with the conv geometry")
    if (not stem and in_scale is None and tile in (None, "patch")
            and patch3_supported(IC, OC, R, S, stride, pad, IH, IW) and IH % 4 == 0
            and (tile == "patch" or _use_patch3(None, "wgrad"))):
        # 3x3 patch kernel (csrc/conv_patch3.hip): one fp32 slab per persistent workgroup
        if (num_cus() + 64) * OC * R * S * IC > ws.numel():  # one slab per CU + the reduction's partials
            raise ValueError("wgrad workspace too small for the patch kernel")
        nsl = C().wgrad_patch3(dy.data_ptr(), x.data_ptr(), ws.data_ptr(), ws.numel(), N, IH, IW, IC, OH, OW, OC, R,
                               S, stride, pad, stream_ptr(),
                               0)  # (honouring cu_reserve here measured slower: profiles/r5_cu_reserve/)
        C().wgrad_reduce(ws.data_ptr(), dw.data_ptr(), OC * KTOT, nsl, float(scale), int(accumulate), stream_ptr())
        return dw
    if isinstance(tile, str):
        raise ValueError("tile='patch' needs a 64->64 3x3 stride-1 wgrad at width 56 without a prologue")
    if stem and OC == 64 and R <= 8 and S <= 8 and tile is None and _stem_wgrad_tile():
        # one 64 x 256 tile per workgroup (csrc/stem_bwd.hip, plain mode): dy read once
        _chk(dy, torch.bfloat16, "dy", N * OH * OW * 64)
        n = C().stem_bwd(0, 0, dy.data_ptr(), 0, 0, 0, x.data_ptr(), ws.data_ptr(), ws.numel(), N, OH, OW, OC, 0, 0,
                         0, 1, 0, IH, IW, R, S, stride, pad, 0, stream_ptr())
        if out_krsc is not None:  # (the image's real channels: x carries them padded to 4)
            icr = out_krsc.numel() // (OC * R * S)
            _chk(out_krsc, torch.float32, "out_krsc", OC * R * S * icr)
            if not 1 <= icr <= IC:
                raise ValueError("out_krsc: (OC, R, S, IC) with IC <= the padded input channels")
            C().wgrad_reduce_gather(ws.data_ptr(), out_krsc.data_ptr(), OC, R, S, icr, n, float(scale),
                                    int(accumulate), stream_ptr())
            return out_krsc
        C().wgrad_reduce(ws.data_ptr(), dw.data_ptr(), OC * KTOT, n, float(scale), int(accumulate), stream_ptr())
        return dw
    if stem:
        bm, bn = 64, 128
    else:
        if OC % 64 or IC % 64:
            raise ValueError("conv_wgrad needs channels % 64 == 0")
        if tile:
            bm, bn = tile
        else:
            t = _tune_table().get(tune_key("wgrad", N * OH * OW, OC, IC, R, stride))
            if t is not None and OC % t[0] == 0 and IC % t[1] == 0:
                bm, bn = t[0], t[1]
                if len(t) > 2 and dma < 0:  # measured operand path (tools/tune_conv.py)
                    dma = int(t[2])
                if len(t) > 3 and rounds is None:  # measured split depth (tools/tune_conv.py --wgrad-rounds)
                    rounds = float(t[3])
            else:
                bm = 128 if OC % 128 == 0 else 64
                bn = 128 if IC % 128 == 0 else 64
    if in_scale is not None:
        _chk(in_scale, torch.float32, "in_scale", IC)
        _chk(in_shift, torch.float32, "in_shift", IC)
    M = N * OH * OW
    if cu_reserve > 0:  # one round over all but cu_reserve CUs (the main stream's small kernels keep a place)
        rounds = min(1.0, 1.0 if rounds is None or rounds <= 0 else float(rounds))
    nsplit, ms = wgrad_splits(M, OC, KTOT, bm, bn, ws.numel(), rounds,
                              cus=num_cus() - cu_reserve if cu_reserve > 0 else None)
    if (nsplit + (min(64, nsplit) if nsplit > 8 else 0)) * OC * KTOT > ws.numel():
        raise ValueError("wgrad workspace too small")
    # one split: the kernel writes the finished gradient itself (no slab, no reduce launch)
    fuse = not stem and (nsplit == 1 or (cnt is not None and nsplit * bm * bn * 4 <= wgrad_fuse_max()))
    if fuse and nsplit > 1:
        _chk(cnt, torch.int32, "cnt")
        if cnt.numel() < (OC // bm) * (KTOT // bn):
            raise ValueError("conv_wgrad: tile counter slice too small")
    region = None
    if (defer is not None and not fuse and (defer.max_slab_bytes is None
                                           or 4 * nsplit * OC * KTOT <= defer.max_slab_bytes)):
        # slabs (+ level-1 partials) in the batch's arena, reduced at its flush
        region = defer.alloc((nsplit + (min(64, nsplit) if nsplit > 8 else 0)) * OC * KTOT)
        if region is not None:
            ws = region
    C().conv_wgrad(STEM if stem else FWD, bm, bn, dy.data_ptr(), x.data_ptr(), ws.data_ptr(), _p(in_scale),
                   _p(in_shift), int(relu_in), N, IH, IW, IC, OH, OW, OC, R, S, stride, pad, KTOT, nsplit, ms,
                   stream_ptr(), int(lds_pad), int(dma), dw.data_ptr() if fuse else 0,
                   cnt.data_ptr() if fuse and cnt is not None else 0, float(scale), int(accumulate))
    if region is not None:
        defer.add(ws, dw, OC * KTOT, nsplit, scale, accumulate)
    elif not fuse:
        C().wgrad_reduce(ws.data_ptr(), dw.data_ptr(), OC * KTOT, nsplit, float(scale), int(accumulate), stream_ptr())
    return dw


def dwfused_supported(C: int, K: int, M: int) -> bool:
    """Geometry of the fused bottleneck-conv3 backward kernel (csrc/conv_dwfused.hip): the 64 -> 256
    conv3 of the 56x56 stage and the 128 -> 512 conv3 of the 28x28 stage (64-pixel tiles), whole
    tiles, 32-bit buffer offsets."""
    return (C, K) in ((64, 256), (128, 512)) and M % 64 == 0 and 2 * M * K < 0xFFFFFF00


def num_cus() -> int:
    """Compute units of the current device (256 on MI355X); 256 when no GPU is visible."""
    global _NUM_CUS
    if _NUM_CUS is None:
        try:
            _NUM_CUS = int(torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count) \
                if torch.cuda.is_available() else 256
        except Exception:
            _NUM_CUS = 256
    return _NUM_CUS


_NUM_CUS = None


def dwfused_grid(C: int, K: int) -> int:
    """Resident workgroups of the fused conv3 backward (csrc/conv_dwfused.hip launches
    occupancy x CUs): 2 per CU for the 64 -> 256 variant, 1 per CU for 128 -> 512."""
    return (2 if (C, K) == (64, 256) else 1) * num_cus()


def dwfused_preferred(C: int, K: int, M: int) -> bool:
    """Schedule policy: the fused conv3 backward only when every resident workgroup walks >=
    ``fuse_dw_min_tiles`` (default 4) tiles -- with fewer, the per-workgroup weight load and slab write
    and the lost wgrad side-stream overlap outweigh the saved traffic (TinyImageNet b512 fused at 2-4
    tiles per workgroup: 86.5k vs 87.2k img/s in round 2, profiles/r2s4_dwfused/; with the round-5
    per-block side forks and the 128-CU reservation its 4-tile layer1 conv3 gains: 104.3k vs 103.7k,
    2 tiles still loses: profiles/r5_side_defer/tiny_knobs_late.txt)."""
    grid = dwfused_grid(C, K)
    return dwfused_supported(C, K, M) and M >= _E().fuse_dw_min_tiles * grid * 64


@_dispatch
def conv_dwfused(g, y3, coeff, wt16, y2, scale2, shift2, mean2, invstd2, bstats2, da, dw, ws, cus: int = 0):
    """Backward of a bottleneck conv3 (1x1 stride 1, C -> K) in one pass (csrc/conv_dwfused.hip):
    dy3 = k1*g + k2*y3 + k3 (BN3-backward apply, ``coeff`` [3, K]) -> data gradient
    ``da`` = [a2 > 0] * conv_transpose(dy3) with the BN2-backward moments into ``bstats2`` (the MASK_Y
    epilogue, a2 = relu(y2*scale2 + shift2)), and weight gradient ``dw`` [K, C] = dy3^T a2 (fp32,
    per-workgroup slabs in ``ws`` + the deterministic split reduction). dy3 and a2 never reach HBM.
    ``cus`` > 0: the persistent grid spans only that many CUs (0: all)."""
    N, H, W, Kc = g.shape
    Cc = y2.shape[-1]
    M = N * H * W
    _chk(g, torch.bfloat16, "g")
    _chk(y3, torch.bfloat16, "y3", g.numel())
    _chk(coeff, torch.float32, "coeff", 3 * Kc)
    _chk(wt16, torch.bfloat16, "wt16", Cc * Kc)
    _chk(y2, torch.bfloat16, "y2", M * Cc)
    _chk(da, torch.bfloat16, "da", M * Cc)
    _chk(dw, torch.float32, "dw", Kc * Cc)
    _chk(ws, torch.float32, "ws")
    nsh2 = _chk_stats(bstats2, "bstats2", Cc)
    for t, nm in ((scale2, "scale2"), (shift2, "shift2"), (mean2, "mean2"), (invstd2, "invstd2")):
        _chk(t, torch.float32, nm, Cc)
    if not dwfused_supported(Cc, Kc, M):
        raise ValueError(f"conv_dwfused: unsupported geometry C={Cc} K={Kc} M={M}")
    n = C().conv_dwfused(g.data_ptr(), y3.data_ptr(), coeff.data_ptr(), wt16.data_ptr(), y2.data_ptr(),
                         scale2.data_ptr(), shift2.data_ptr(), mean2.data_ptr(), invstd2.data_ptr(), da.data_ptr(),
                         bstats2.data_ptr(), ws.data_ptr(), ws.numel(), M, Kc, Cc, nsh2, stream_ptr(), int(cus))
    C().wgrad_reduce(ws.data_ptr(), dw.data_ptr(), Kc * Cc, n, 1.0, 0, stream_ptr())
    return da


# --------------------------------------------------------------------------------------
# batch norm / elementwise
# --------------------------------------------------------------------------------------
@_dispatch
def bn_finalize(stats, count, gamma, beta, eps, momentum, running_mean, running_var, scale, shift,
                save_mean, save_invstd):
    Cc = scale.numel()
    C().bn_finalize(stats.data_ptr(), _nsh(stats, Cc), Cc, float(count), _p(gamma), _p(beta), float(eps), float(momentum),
                    _p(running_mean), _p(running_var), scale.data_ptr(), shift.data_ptr(), _p(save_mean),
                    _p(save_invstd), stream_ptr())


@_dispatch
def bn_eval_coeff(gamma, beta, eps, running_mean, running_var, scale, shift):
    C().bn_eval_coeff(scale.numel(), _p(gamma), _p(beta), float(eps), running_mean.data_ptr(),
                      running_var.data_ptr(), scale.data_ptr(), shift.data_ptr(), stream_ptr())


@_dispatch
def channel_stats(y, stats):
    Cc = y.shape[-1]
    _chk(y, torch.bfloat16, "y")
    nsh = _chk_stats(stats, "stats", Cc)
    C().channel_stats(y.data_ptr(), y.numel() // Cc, Cc, stats.data_ptr(), nsh, stream_ptr())


@_dispatch
def bn_apply(y, scale, shift, out, *, res=None, res_scale=None, res_shift=None, relu=True, mbits=None, fin=None,
             res_fin=None):
    """out = relu(y*scale + shift [+ res | + res*res_scale + res_shift]); ``mbits`` (uint8,
    numel/8): also store the 1-bit ReLU mask (bit j of byte i = element 8i+j > 0) for backward.
    ``fin`` / ``res_fin`` (:class:`BnFin`, mode FWD): the forward finalize of the BN giving scale / shift
    (res_scale / res_shift) is done inside this launch (the bn_finalize launch it replaces, bit for bit;
    its outputs are stored on the way)."""
    Cc = y.shape[-1]
    _chk(y, torch.bfloat16, "y")
    _chk(out, torch.bfloat16, "out", y.numel())
    mode = 0
    if res is not None:
        _chk(res, torch.bfloat16, "res", y.numel())
        mode = 2 if res_scale is not None else 1
    if mbits is not None:
        _chk(mbits, torch.uint8, "mbits", y.numel() // 8)
    fins = []
    for f in (fin, res_fin if mode == 2 else None):
        if f is not None and f.desc is None:
            f.run()
            f = None
        fins.append(f.ptr() if f else 0)
    if res_fin is not None and mode != 2:
        res_fin.run()
    C().bn_apply(y.data_ptr(), scale.data_ptr(), shift.data_ptr(), _p(res), _p(res_scale), _p(res_shift),
                 out.data_ptr(), y.numel(), Cc, mode, int(relu), _p(mbits), stream_ptr(), *fins)
    return out



@_dispatch
def bn_bwd_reduce(dout, y, mean, invstd, stats, *, mask_mode, mref=None, scale=None, shift=None):
    Cc = y.shape[-1]
    _chk(dout, torch.bfloat16, "dout", y.numel())
    _chk(y, torch.bfloat16, "y")
    nsh = _chk_stats(stats, "stats", Cc)
    if mask_mode == MASK_OUT:
        _chk(mref, torch.bfloat16, "mref", y.numel())
    C().bn_bwd_reduce(dout.data_ptr(), _p(mref), y.data_ptr(), _p(scale), _p(shift), mean.data_ptr(),
                      invstd.data_ptr(), y.numel() // Cc, Cc, stats.data_ptr(), nsh, mask_mode, stream_ptr())


@_dispatch
def bn_bwd_coeff(stats, count, gamma, mean, invstd, coeff, dgamma=None, dbeta=None, accumulate=False):
    Cc = mean.numel()
    C().bn_bwd_coeff(stats.data_ptr(), _nsh(stats, Cc), Cc, float(count), _p(gamma), mean.data_ptr(), invstd.data_ptr(),
                     coeff.data_ptr(), _p(dgamma), _p(dbeta), int(accumulate), stream_ptr())


@_dispatch
def bn_bwd_apply(dout, y, coeff, dy, *, mask_mode, mref=None, scale=None, shift=None, gout=None, fin=None):
    """dy = k1*g + k2*y + k3 with g = dout masked by ``mask_mode``. ``fin`` (:class:`BnFin`, mode BWD):
    the coefficients are finalized inside this launch from the BN's moment shards (the bn_bwd_coeff
    launch it replaces, bit for bit; ``coeff`` / dgamma / dbeta are stored on the way)."""
    Cc = y.shape[-1]
    _chk(dy, torch.bfloat16, "dy", y.numel())
    if gout is not None:
        _chk(gout, torch.bfloat16, "gout", y.numel())
    if fin is not None and fin.desc is None:  # (no device descriptor: the standalone launch first)
        fin.run()
        fin = None
    C().bn_bwd_apply(dout.data_ptr(), _p(mref), y.data_ptr(), _p(scale), _p(shift), coeff.data_ptr(),
                     dy.data_ptr(), _p(gout), y.numel(), Cc, mask_mode, stream_ptr(), fin.ptr() if fin else 0)


@_dispatch
def bn_bwd_apply2(g, y1, coeff1, dy1, y2, coeff2, dy2, fin1=None, fin2=None):
    """Two unmasked BN-backward applies sharing the gradient g (one read of g):
    dy1 = k1*g + k2*y1 + k3 (coeff1), dy2 likewise with y2 / coeff2; ``fin1`` / ``fin2`` as in
    :func:`bn_bwd_apply`."""
    Cc = y1.shape[-1]
    for t, nm in ((g, "g"), (y1, "y1"), (dy1, "dy1"), (y2, "y2"), (dy2, "dy2")):
        _chk(t, torch.bfloat16, nm, y1.numel())
    _chk(coeff1, torch.float32, "coeff1", 3 * Cc)
    _chk(coeff2, torch.float32, "coeff2", 3 * Cc)
    fins = []
    for f in (fin1, fin2):
        if f is not None and f.desc is None:
            f.run()
            f = None
        fins.append(f.ptr() if f else 0)
    C().bn_bwd_apply2(g.data_ptr(), y1.data_ptr(), coeff1.data_ptr(), dy1.data_ptr(), y2.data_ptr(),
                      coeff2.data_ptr(), dy2.data_ptr(), y1.numel(), Cc, stream_ptr(), *fins)


@_dispatch
def maxpool_fwd(x, out, arg, *, K=3, stride=2, pad=1, scale=None, shift=None, relu=True, ymax=None, fin=None):
    """out = max over windows of relu(x*scale + shift), arg = window index of the max; ``ymax``
    (optional) = the raw x at the argmax (the stem BN backward reduces over pooled positions).
    ``fin`` (:class:`BnFin`, mode FWD): the stem BN's forward finalize, done inside this launch."""
    N, H, W, Cc = x.shape
    _, P, Q, _ = out.shape
    _chk(x, torch.bfloat16, "x")
    _chk(out, torch.bfloat16, "out")
    _chk(arg, torch.uint8, "arg", out.numel())
    if ymax is not None:
        _chk(ymax, torch.bfloat16, "ymax", out.numel())
    if fin is not None and (fin.desc is None or scale is None):
        fin.run()
        fin = None
    C().maxpool_fwd(x.data_ptr(), _p(scale), _p(shift), out.data_ptr(), arg.data_ptr(), _p(ymax), N, H, W, Cc, P, Q,
                    K, stride, pad, int(relu), stream_ptr(), fin.ptr() if fin else 0)


@_dispatch
def maxpool_bwd(dout, arg, dx, *, K=3, stride=2, pad=1):
    N, H, W, Cc = dx.shape
    _, P, Q, _ = dout.shape
    _chk(dout, torch.bfloat16, "dout")
    _chk(arg, torch.uint8, "arg", dout.numel())
    _chk(dx, torch.bfloat16, "dx")
    C().maxpool_bwd(dout.data_ptr(), arg.data_ptr(), dx.data_ptr(), N, H, W, Cc, P, Q, K, stride, pad, stream_ptr())


def _pool_bn_bwd_check(dpool, arg, y, K, stride):
    N, H, W, Cc = y.shape
    _chk(dpool, torch.bfloat16, "dpool")
    _chk(arg, torch.uint8, "arg", dpool.numel())
    _chk(y, torch.bfloat16, "y")
    if dpool.shape[0] != N or dpool.shape[3] != Cc:
        raise ValueError("pool_bn_bwd: dpool / y shapes disagree")
    if Cc % 8 or 256 % (Cc // 8) or (K + stride - 1) // stride > 2:
        raise ValueError("pool_bn_bwd: unsupported channel count / pool geometry")
    return N, H, W, Cc, dpool.shape[1], dpool.shape[2]


def pool_bn_bwd_supported(C: int, K: int, stride: int) -> bool:
    return C % 8 == 0 and 256 % (C // 8) == 0 and (K + stride - 1) // stride <= 2


@_dispatch
def pool_bn_bwd_reduce(dpool, arg, y, scale, shift, mean, invstd, stats, *, K=3, stride=2, pad=1):
    """BN-backward reduce of the stem BN with the max-pool backward folded in: g = maxpool_bwd(dpool)
    masked by relu(y*scale+shift) > 0; stats += [sum g, sum g*xhat]. The pooled-gradient
    tensor at the pool input resolution is never materialised."""
    N, H, W, Cc, Pp, Q = _pool_bn_bwd_check(dpool, arg, y, K, stride)
    nsh = _chk_stats(stats, "stats", Cc)
    C().pool_bn_bwd(dpool.data_ptr(), arg.data_ptr(), y.data_ptr(), scale.data_ptr(), shift.data_ptr(),
                    mean.data_ptr(), invstd.data_ptr(), 0, 0, stats.data_ptr(), nsh, N, H, W, Cc, Pp, Q, K,
                    stride, pad, 0, stream_ptr())


@_dispatch
def pool_bn_bwd_apply(dpool, arg, y, scale, shift, coeff, dy, *, K=3, stride=2, pad=1):
    """dy = k1*g + k2*y + k3 with g recomputed as in ``pool_bn_bwd_reduce``."""
    N, H, W, Cc, Pp, Q = _pool_bn_bwd_check(dpool, arg, y, K, stride)
    _chk(dy, torch.bfloat16, "dy", y.numel())
    C().pool_bn_bwd(dpool.data_ptr(), arg.data_ptr(), y.data_ptr(), scale.data_ptr(), shift.data_ptr(),
                    coeff.data_ptr(), coeff.data_ptr() + 4 * Cc, coeff.data_ptr() + 8 * Cc, dy.data_ptr(), 0, 1,
                    N, H, W, Cc, Pp, Q, K, stride, pad, 1, stream_ptr())


def stem_bwd_supported(C: int, K: int, stride: int, R: int, S: int) -> bool:
    """Geometry of the fused stem backward (csrc/stem_bwd.hip): 64 stem channels, <= 8x8 taps,
    pooling windows that cover a pixel at most twice per dimension."""
    return C == 64 and R <= 8 and S <= 8 and (K + stride - 1) // stride <= 2


@_dispatch
def stem_bwd_fused(dpool, arg, y, scale, shift, coeff, x4, dw, ws, *, K=3, stride=2, pad=1, R=7, S=7,
                   conv_stride=2, conv_pad=3):
    """Stem backward in one pass (csrc/stem_bwd.hip): dy = BN-backward apply of the max-pool
    backward of ``dpool`` (argmax ``arg``, ReLU mask from ``y*scale + shift``) -- never stored -- and
    the stem weight gradient ``dw`` [C, 8*8*4] fp32 (the stem's padded tap layout) = dy^T im2col(x4),
    through per-workgroup slabs in ``ws`` + the deterministic split reduction. Replaces
    ``pool_bn_bwd_apply`` + ``conv_wgrad(..., stem=True)``."""
    N, H, W, Cc, Pp, Q = _pool_bn_bwd_check(dpool, arg, y, K, stride)
    _chk(x4, torch.bfloat16, "x4")
    _chk(coeff, torch.float32, "coeff", 3 * Cc)
    _chk(scale, torch.float32, "scale", Cc)
    _chk(shift, torch.float32, "shift", Cc)
    _chk(dw, torch.float32, "dw", Cc * 256)
    _chk(ws, torch.float32, "ws")
    Nx, IH, IW, C4 = x4.shape
    if Nx != N or C4 != 4 or conv_out_hw(IH, IW, R, S, conv_stride, conv_pad) != (H, W):
        raise ValueError("stem_bwd_fused: image / stem output shapes disagree")
    if not stem_bwd_supported(Cc, K, stride, R, S):
        raise ValueError("stem_bwd_fused: unsupported geometry")
    n = C().stem_bwd(dpool.data_ptr(), arg.data_ptr(), y.data_ptr(), scale.data_ptr(), shift.data_ptr(),
                     coeff.data_ptr(), x4.data_ptr(), ws.data_ptr(), ws.numel(), N, H, W, Cc, Pp, Q, K, stride, pad,
                     IH, IW, R, S, conv_stride, conv_pad, 1, stream_ptr())
    C().wgrad_reduce(ws.data_ptr(), dw.data_ptr(), Cc * 256, n, 1.0, 0, stream_ptr())
    return dw


@_dispatch
def avgpool_fwd(x, out):
    N, H, W, Cc = x.shape
    _chk(x, torch.bfloat16, "x")
    _chk(out, torch.bfloat16, "out", N * Cc)
    C().avgpool_fwd(x.data_ptr(), out.data_ptr(), N, H * W, Cc, stream_ptr())


@_dispatch
def avgpool_bwd(dout, dx):
    N, H, W, Cc = dx.shape
    _chk(dout, torch.bfloat16, "dout", N * Cc)
    _chk(dx, torch.bfloat16, "dx")
    C().avgpool_bwd(dout.data_ptr(), dx.data_ptr(), N, H * W, Cc, stream_ptr())


@_dispatch
def softmax_ce(logits, labels, dlogits=None, loss_out=None, stats=None, smoothing=0.0, grad_scale=1.0,
               labels2=None, lam=None):
    """Fused softmax cross-entropy (+ label smoothing) with dlogits, per-row loss, device-side
    loss-sum / correct counters. ``labels2`` [B] int64 + ``lam`` fp32[1] device (CutMix): the target
    is lam * onehot(labels) + (1 - lam) * onehot(labels2), smoothed on top."""
    B, Cc = logits.shape
    if logits.dtype not in (torch.float32, torch.bfloat16) or not logits.is_contiguous():
        raise TypeError("logits must be contiguous fp32/bf16")
    _chk(labels, torch.int64, "labels", B)
    if dlogits is not None:
        _chk(dlogits, logits.dtype, "dlogits", B * Cc)
    if stats is not None:
        _chk(stats, torch.float64, "stats", 2)
    if (labels2 is None) != (lam is None):
        raise ValueError("labels2 and lam come together")
    if labels2 is not None:
        _chk(labels2, torch.int64, "labels2", B)
        _chk(lam, torch.float32, "lam", 1)
    C().softmax_ce(logits.data_ptr(), int(logits.dtype == torch.bfloat16), labels.data_ptr(), _p(dlogits),
                   _p(loss_out), _p(stats), B, Cc, float(smoothing), float(grad_scale), _p(labels2), _p(lam),
                   stream_ptr())


def dropout_threshold(p_drop: float) -> Tuple[int, float]:
    """(thresh, 1/keep) for a Philox draw u32 < thresh keeping an element with prob 1 - p_drop."""
    keep = 1.0 - float(p_drop)
    if not 0.0 < keep <= 1.0:
        raise ValueError("dropout probability must be in [0, 1)")
    return min(0xFFFFFFFF, int(round(keep * 4294967296.0))), 1.0 / keep


def head_splitk(M: int, N: int, K: int, ws_elems: int) -> int:
    """Split-K depth of a head GEMM: long-K shapes with few 64 x 64 tiles (< 192: the fc forward at
    TinyImageNet's batch 512 / 200 classes has 32) split K so ~256 workgroups run, >= 2 k-stages each."""
    tiles = -(-M // 64) * -(-N // 64)
    kst = -(-K // 128)
    if not _E().head_splitk or tiles >= 192 or kst < 4 or ws_elems < 2 * M * N:
        return 1
    return max(1, min(kst // 2, max(2, 256 // tiles), 64, ws_elems // (M * N)))


@_dispatch
def small_gemm(A, B, out, *, ta=False, tb=False, M, N, K, alpha=1.0, bias=None, accumulate=False,
               dropout=None, ws=None):
    """out[M, N] (fp32 / bf16) = alpha * A(m, k) B(k, n) (+ bias[n]) (+ out) on MFMA (csrc/head_ops.hip).
    A: ``ta`` False -> [M, K], True -> [K, M]; B: ``tb`` False -> [N, K], True -> [K, N] (bf16, contiguous).
    ``dropout``: (operand "A" | "B", p, seed, offset) -- Philox mask on that operand's elements; ``offset``
    an int or an int32[1] device tensor (read by the kernel: a replayed graph draws a new mask each step).
    ``ws``: fp32 workspace enabling split-K for long-K / few-tile shapes (:func:`head_splitk`)."""
    _chk(A, torch.bfloat16, "A", M * K)
    _chk(B, torch.bfloat16, "B", N * K)
    if out.dtype not in (torch.float32, torch.bfloat16) or out.numel() != M * N or not out.is_contiguous():
        raise ValueError("out must be a contiguous fp32/bf16 [M, N]")
    bf = bh = None
    if bias is not None:
        if bias.numel() != N:
            raise ValueError("bias must have N elements")
        bf, bh = (bias, None) if bias.dtype == torch.float32 else (None, bias)
    drop, seed, off, thr, inv, offd = 0, 0, 0, 0, 1.0, None
    if dropout is not None:
        which, pd, seed, off = dropout
        drop = 1 if which == "A" else 2
        thr, inv = dropout_threshold(pd)
        if isinstance(off, torch.Tensor):
            _chk(off, torch.int32, "dropout offset", 1)
            off, offd = 0, off
    lda = M if ta else K
    ldb = N if tb else K
    sk = 1
    if ws is not None:
        _chk(ws, torch.float32, "ws")
        sk = head_splitk(M, N, K, ws.numel())
    C().small_gemm(int(ta), int(tb), int(out.dtype == torch.float32), drop, A.data_ptr(), B.data_ptr(), out.data_ptr(),
                   _p(bf), _p(bh), M, N, K, lda, ldb, N, float(alpha), int(accumulate), int(seed) & ((1 << 64) - 1),
                   int(off) & 0xFFFFFFFF, thr, float(inv), _p(offd), stream_ptr(), ws.data_ptr() if sk > 1 else 0, sk)
    return out


@_dispatch
def colsum(x, out, accumulate=False):
    """out[n] (+)= sum_m x[m, n] (bf16 -> fp32, fixed order): the fc bias gradient."""
    M, N = x.shape
    _chk(x, torch.bfloat16, "x")
    _chk(out, torch.float32, "out", N)
    C().colsum(x.data_ptr(), out.data_ptr(), M, N, int(accumulate), stream_ptr())
    return out


@_dispatch
def dropout(x, y, p, seed, offset):
    """y = x * Philox mask (keep 1-p, scale 1/(1-p)); the same (seed, offset) regenerate the mask."""
    _chk(x, torch.bfloat16, "x")
    _chk(y, torch.bfloat16, "y", x.numel())
    thr, inv = dropout_threshold(p)
    offd = None
    if isinstance(offset, torch.Tensor):
        _chk(offset, torch.int32, "offset", 1)
        offset, offd = 0, offset
    C().dropout(x.data_ptr(), y.data_ptr(), x.numel(), int(seed) & ((1 << 64) - 1), int(offset) & 0xFFFFFFFF, thr,
                float(inv), _p(offd), stream_ptr())
    return y


@_dispatch
def sgd_step(p, g, v, p16=None, *, lr, momentum, dampening=0.0, weight_decay=0.0, nesterov=False, first=False,
             grad_scale_ptr=None, grad_scale=1.0, hyper=None):
    """PyTorch-SGD semantics. ``hyper`` (fp32[1] device tensor) overrides ``lr`` at run time."""
    n = p.numel()
    _chk(p, torch.float32, "p")
    _chk(g, torch.float32, "g", n)
    _chk(v, torch.float32, "v", n)
    if p16 is not None:
        _chk(p16, torch.bfloat16, "p16", n)
    C().sgd(p.data_ptr(), g.data_ptr(), v.data_ptr(), _p(p16), n, _p(hyper), float(lr), float(momentum), float(dampening),
            float(weight_decay), int(nesterov), int(first), _p(grad_scale_ptr), float(grad_scale), stream_ptr())


LARS_MAX_BLOCKS = 64  # csrc/nn_ops.hip kLarsMaxBlocks


@_dispatch
def lars_scale(p, g, seg_off, seg_len, adapt, norms, *, grad_scale, eta, weight_decay, max_len):
    """LARS pre-scaling of the flat gradient in place (then ``sgd_step`` with wd=0): per segment
    trust = eta*|w|/(|gs*g| + wd*|w|); adapted segments get g = trust*(gs*g + wd*w), the others gs*g.
    ``seg_off`` / ``seg_len`` / ``adapt``: int32 device tensors [nseg]; ``norms``: fp64 [nseg*64*2] scratch
    (one partial pair per segment and block, summed in fixed block order: bit-reproducible)."""
    n = p.numel()
    _chk(p, torch.float32, "p")
    _chk(g, torch.float32, "g", n)
    nseg = seg_off.numel()
    for t, nm in ((seg_off, "seg_off"), (seg_len, "seg_len"), (adapt, "adapt")):
        _chk(t, torch.int32, nm, nseg)
    _chk(norms, torch.float64, "norms", LARS_MAX_BLOCKS * 2 * nseg)
    C().lars_scale(p.data_ptr(), g.data_ptr(), seg_off.data_ptr(), seg_len.data_ptr(), adapt.data_ptr(), nseg,
                   int(max_len), norms.data_ptr(), float(grad_scale), float(eta), float(weight_decay), stream_ptr())


@_dispatch
def adam_step(p, g, m, v, p16=None, *, lr, beta1, beta2, eps, weight_decay, decoupled, step,
              grad_scale_ptr=None, grad_scale=1.0, hyper=None):
    """Adam / AdamW. ``hyper`` (fp32[3] device: lr, 1-b1^t, 1-b2^t) overrides lr/step at run time."""
    n = p.numel()
    for t, nm in ((p, "p"), (g, "g"), (m, "m"), (v, "v")):
        _chk(t, torch.float32, nm, n)
    bc1 = 1.0 - beta1 ** step
    bc2 = 1.0 - beta2 ** step
    C().adam(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), _p(p16), n, _p(hyper), float(lr), float(beta1),
             float(beta2), float(eps), float(weight_decay), int(decoupled), float(bc1), float(bc2),
             _p(grad_scale_ptr), float(grad_scale), stream_ptr())


@_dispatch
def global_norm_clip_factor(g, max_norm, work):
    """work: fp32[4] scratch (work[0:2] holds the fp64 sum of squares); returns work[2:4] =
    (factor, norm) on device (no host sync)."""
    work.zero_()
    C().sumsq(g.data_ptr(), g.numel(), work.data_ptr(), stream_ptr())
    C().clip_factor(work.data_ptr(), float(max_norm), work[2:].data_ptr(), stream_ptr())
    return work[2:3]


@_dispatch
def sumsq_accum(g, work):
    """work[0:2] (viewed as one fp64) += sum of squares of the fp32 tensor ``g`` (no zeroing)."""
    _chk(g, torch.float32, "g")
    _chk(work, torch.float32, "work")
    C().sumsq(g.data_ptr(), g.numel(), work.data_ptr(), stream_ptr())


@_dispatch
def clip_factor(work, max_norm):
    """work[2:4] = (min(1, max_norm / (norm + 1e-6)), norm) from the fp64 sum of squares in work[0:2]."""
    C().clip_factor(work.data_ptr(), float(max_norm), work[2:].data_ptr(), stream_ptr())
    return work[2:3]


@_dispatch
def normalize_u8(img, out, mean, std, flip=None):
    N, H, W, Cin = img.shape
    _chk(img, torch.uint8, "img")
    _chk(out, torch.bfloat16, "out", N * H * W * 4)
    if flip is not None:
        _chk(flip, torch.uint8, "flip", N)
    C().normalize_u8(img.data_ptr(), out.data_ptr(), _p(flip), N, H, W, Cin, float(mean[0]), float(mean[1]),
                     float(mean[2]), float(std[0]), float(std[1]), float(std[2]), stream_ptr())


@_dispatch
def augment_u8(img, out, boxes, mean, std, flip=None, perm=None, mixbox=None):
    """uint8 NHWC -> bf16 NHWC4: per-sample crop box [N,4] (y0, x0, h, w; fp32) bilinear-resized to
    out's H x W, optional flip [N] uint8, normalised. CutMix: ``perm`` [N] int32 + ``mixbox`` int32
    [y0, y1, x0, x1] (output coordinates; empty box = no mixing) paste sample perm[n]'s augmented
    pixels into the box."""
    N, Hin, Win, Cin = img.shape
    _, Ho, Wo, C4 = out.shape
    _chk(img, torch.uint8, "img")
    _chk(out, torch.bfloat16, "out", N * Ho * Wo * 4)
    _chk(boxes, torch.float32, "boxes", N * 4)
    if flip is not None:
        _chk(flip, torch.uint8, "flip", N)
    if (perm is None) != (mixbox is None):
        raise ValueError("perm and mixbox come together")
    if perm is not None:
        _chk(perm, torch.int32, "perm", N)
        _chk(mixbox, torch.int32, "mixbox", 4)
    C().augment_u8(img.data_ptr(), out.data_ptr(), boxes.data_ptr(), _p(flip), N, Hin, Win, Cin, Ho, Wo,
                   float(mean[0]), float(mean[1]), float(mean[2]), float(std[0]), float(std[1]), float(std[2]),
                   _p(perm), _p(mixbox), stream_ptr())


@_dispatch
def weight_prep(master, wbuf, desc_dev, nlayers):
    """bf16 forward (KRSC) and dgrad (CRSK) weight copies from the flat fp32 master -- or from a
    flat bf16 parameter copy of the same layout (ZeRO: the all-gathered ``param16``)."""
    if master.dtype == torch.bfloat16:
        C().weight_prep16(master.data_ptr(), wbuf.data_ptr(), desc_dev.data_ptr(), nlayers, stream_ptr())
    else:
        C().weight_prep(master.data_ptr(), wbuf.data_ptr(), desc_dev.data_ptr(), nlayers, stream_ptr())


@_dispatch
def cast_f32_bf16(x, y):
    _chk(x, torch.float32, "x")
    _chk(y, torch.bfloat16, "y", x.numel())
    C().cast_f32_bf16(x.data_ptr(), y.data_ptr(), x.numel(), stream_ptr())


def pack_mask_bits(x: torch.Tensor) -> torch.Tensor:
    """uint8 [numel/8]: bit j of byte i = (x.flat[8i+j] > 0) — the layout bn_apply(mbits=) writes."""
    b = (x.reshape(-1, 8) > 0).to(torch.uint8)
    w = torch.tensor([1, 2, 4, 8, 16, 32, 64, 128], dtype=torch.uint8, device=x.device)
    return (b * w).sum(1, dtype=torch.int32).to(torch.uint8)


def unpack_mask_bits(bits: torch.Tensor, shape) -> torch.Tensor:
    w = torch.tensor([1, 2, 4, 8, 16, 32, 64, 128], dtype=torch.uint8, device=bits.device)
    return ((bits.view(-1, 1) & w) != 0).reshape(shape)
