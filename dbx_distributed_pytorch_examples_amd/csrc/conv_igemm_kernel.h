// NHWC bf16 implicit-GEMM convolution on CDNA4 MFMA (v_mfma_f32_16x16x32_bf16).
//
// Replaces the cuDNN/MIOpen conv kernels the reference reaches through torchvision
// (SURVEY.md §2.4 K1-K5). One kernel family, three problem mappings:
//
//   FWD    Y[m=(n,oh,ow)][k]  = sum_{r,s,c} X[n][oh*st-pad+r][ow*st-pad+s][c] * W[k][r][s][c]
//   DGRAD  dX[m=(n,h,w)][c]   = sum_{r,s,k} dY[n][(h+pad-r)/st][(w+pad-s)/st][k] * Wt[c][r][s][k]
//          (transposed gather: a tap contributes only where (h+pad-r) % st == 0)
//   STEM   the 7x7 C=3 stem with the image padded to 4 channels: a "tap" is one filter row r
//          and its 8 pixels x 4 channels (64 contiguous bytes of an input row); K = 8 x 32.
//
// GEMM view: M = output pixels, N = output channels, K = taps x input channels. Both operands are
// K-contiguous (NHWC activations, KRSC weights), so every lane loads 16 contiguous bytes and the
// MFMA fragments come straight out of LDS with ds_read_b128 (XOR-swizzled: conflict-free).
//
// Fusions (the reason this exists rather than MIOpen — the reference profile spends more time
// in BatchNorm/ReLU/add passes than in the convolutions, profiles/r1_torch_reference):
//   * prologue: BN-apply (+ReLU) of the PREVIOUS layer on the A operand while staging it
//     (y_prev * scale[c] + shift[c], max 0), so BN outputs are never materialised;
//   * epilogue: per-output-channel sum / sum-of-squares for THIS layer's BN, from the fp32
//     accumulators: fp32 per-tile partials added into sharded fp64 slabs (fp64 atomics: the
//     sum of fp32 partials is exact in fp64 for any realistic spread, so the result does not
//     depend on the order the tiles finish in -> bit-reproducible training);
//   * epilogue: accumulate into the existing output (dX of a block = dgrad(conv1) + dgrad(ds)).
//
// Tiles: BM x BN x 64, 256 threads = 2x2 waves, double-buffered LDS with register staging
// (the prologue needs the data in registers anyway), one barrier per K block, XCD-aware
// tile order (A-sharing tiles adjacent -> same XCD L2).
#pragma once
#include <type_traits>
#include "common.h"
#include "abi.h"
#include "bn_fin.h"

namespace dbx {

enum ConvMode { FWD = 0, DGRAD = 1, STEM = 2, FWD_PATCH = 3, DGRAD_PATCH = 4 };

// LDS image swizzle of a [rows][BK] bf16 operand stage: the 16-B chunk ch of row `row` sits at chunk
// position ch ^ fswz<BK>(row). BK = 64 (128-B rows): (row >> 1) & 7. BK = 32 (64-B rows, four rows
// per 256-B bank window): chunk bit 1 flipped for rows 8-15 of every 16 -- each ds_read_b128 lane
// group (rows 0-3 and 12-15 at one chunk, rows 4-11 at the next) then covers 16 distinct 16-B slots
// of the window: conflict-free (the four row quads map to chunk xors 0, 0, 2, 2, so {c, c^2, c^1,
// c^3} are distinct for every c).
template <int BK>
__device__ __forceinline__ int fswz(int row) {
  return BK == 64 ? ((row >> 1) & 7) : (((row >> 3) & 1) << 1);
}


// ---- epilogue (shared by igemm_kernel and the 3x3 patch kernel) ---------------------------------
// acc: this wave's (BM/WM) x (BN/WN) accumulators of the tile starting at output row m0 / channel n0;
// lds: >= BM*(BN+8) bf16 + the reduction scratch; tm: the tile's M index (statistics shard);
// shard: the BN-backward statistics shard selector. Ends with the LDS free for reuse after a barrier.
template <int BM, int BN, int WM, int WN, int MODE, bool STATS, bool ACCUM, int EPI, int EGMAX = 4>
__device__ __forceinline__ void igemm_epilogue(const IGemmArgs& a, f32x4 (&acc)[BM / (16 * WM)][BN / (16 * WN)],
                                               bf16* lds, const int m0, const int n0, const int tm,
                                               const int shard) {
  constexpr int NT = 64 * WM * WN, NW = WM * WN;
  constexpr int TM = BM / (16 * WM), TN = BN / (16 * WN);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wm = wid / WN, wn = wid % WN;
  const u32x4 zero4 = {0u, 0u, 0u, 0u};
  // acc[i][j][r] (C^T): pixel row = wm*BM/WM + i*16 + (lane&15), channel = wn*BN/WN + j*16 + (lane>>4)*4 + r
  // staged bf16 through LDS ([BM][BN+8]: the 8-byte writes of a wave hit each bank 4 times, the
  // minimum for 512 B) and re-read as 16-byte row chunks for coalesced global stores
  static_assert(!(STATS && EPI), "forward BN statistics and BN-backward epilogues are exclusive");
  bf16* sC = lds;  // [BM][BN+8]
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int row = wm * (BM / WM) + i * 16 + (lane & 15);
      const int col = wn * (BN / WN) + j * 16 + (lane >> 4) * 4;
      *reinterpret_cast<uint2*>(sC + row * (BN + 8) + col) =
          uint2{pack2(acc[i][j][0], acc[i][j][1]), pack2(acc[i][j][2], acc[i][j][3])};
    }
  __syncthreads();
  constexpr int CPR = BN / 8;  // 16B chunks per output row; a thread's chunk column is fixed
  const int ccol = tid % CPR;
  // per-thread partial sums of this thread's 8 channels: STATS: sum y, sum y^2 of the stored
  // (bf16-rounded) outputs; EPI: BN-backward raw moments
  float bs[8], bq1[8], bq2[8];
  // accumulated in packed fp32 (v_pk_add_f32 / v_pk_fma_f32: 2 channels per instruction):
  // ps2 = sum, pq2 = sum of squares (STATS) or sum g*y (EPI), pr2 = sum g*y2 (EPI)
  f32x2 ps2[4], pq2[4], pr2[4];
  f32x4 e_m1[2], e_i1[2], e_m2[2], e_i2[2], e_sc[2], e_sh[2];
  const bool has2 = EPI > 0 && a.ybn2 != nullptr;  // wave-uniform: second BN (downsample branch)
  if constexpr (EPI > 0) {
    // vector loads of the per-channel coefficients; absent ones read a valid stand-in (no branch)
    int c0 = n0 + ccol * 8;
    // opaque to the optimiser: in a persistent caller these tile-invariant loads would otherwise be
    // hoisted out of its tile loop and hold 48 VGPRs across the MFMA loop
    asm volatile("" : "+v"(c0));
    const float* m2 = has2 ? a.mean2 : a.mean1;
    const float* i2 = has2 ? a.inv2 : a.inv1;
    const float* sc = (EPI == 2) ? a.bsc : a.mean1;
    const float* sh = (EPI == 2) ? a.bsh : a.inv1;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      e_m1[h] = *reinterpret_cast<const f32x4*>(a.mean1 + c0 + 4 * h);
      e_i1[h] = *reinterpret_cast<const f32x4*>(a.inv1 + c0 + 4 * h);
      e_m2[h] = *reinterpret_cast<const f32x4*>(m2 + c0 + 4 * h);
      e_i2[h] = *reinterpret_cast<const f32x4*>(i2 + c0 + 4 * h);
      e_sc[h] = *reinterpret_cast<const f32x4*>(sc + c0 + 4 * h);
      e_sh[h] = *reinterpret_cast<const f32x4*>(sh + c0 + 4 * h);
    }
#pragma unroll
    for (int h = 0; h < 4; ++h) ps2[h] = pq2[h] = pr2[h] = f32x2{0.f, 0.f};
  }
  // Epilogue in groups of EG rows per thread, in three straight-line phases: (1) every global load
  // of the group (residual addend, mask reference, BN inputs) — rows past M and absent addends read
  // a valid stand-in address instead of branching; (2) all arithmetic; (3) all stores. No load is
  // consumed after a store is issued and no load sits under divergent control flow, so hipcc waits
  // with counted vmcnt instead of draining the queue (stores count in vmcnt too) once per row.
  constexpr int NIT = BM * CPR / NT;
  // EGMAX (default 4): BN epilogues hold 4-5 vectors per row: stay clear of spills
  constexpr int EG = NIT < EGMAX ? NIT : EGMAX;
  const bool sub_geom = MODE == DGRAD && (a.osub > 1 || (ACCUM && a.add_sub > 1));  // wave-uniform
  const bool tail = m0 + BM > a.M;                                                  // wave-uniform
  // one group of G rows per thread (G = EG, and a final NIT % EG group when EG does not tile NIT)
  auto group = [&](const int g0, auto gcount) __attribute__((always_inline)) {
    constexpr int G = decltype(gcount)::value;
    u32x4 vv[G], va[G], vy[G], vy2[G], va2[G];
    unsigned vm[G];  // EPI 1: this chunk's 8 mask bits
    size_t ee[G];
    bool ok[G], has_add[G];
#pragma unroll
    for (int k = 0; k < G; ++k) {
      const int row = (tid + (g0 + k) * NT) / CPR;
      const int m = m0 + row;
      ok[k] = m < a.M;
      const int mc = ok[k] ? m : m0;  // m0 < M for every launched tile
      vv[k] = *reinterpret_cast<const u32x4*>(sC + row * (BN + 8) + ccol * 8);
      size_t pix = (size_t)mc;
      int ph = 0, pw = 0, nimg = 0;
      if (sub_geom) {
        const int ohw = a.OH * a.OW;
        const int n = mdiv_or(mc, a.mag_ohw, ohw), pq = mc - n * ohw;
        const int i = mdiv_or(pq, a.mag_ow, a.OW), j = pq - i * a.OW;
        ph = i * a.osub + a.oph; pw = j * a.osub + a.opw;
        nimg = n;
        pix = ((size_t)n * a.FH + ph) * a.FW + pw;
      }
      const size_t e = pix * a.OC + n0 + ccol * 8;
      DBX_DCHECK(!ok[k] || e + 8 <= (size_t)(sub_geom ? (size_t)a.N * a.FH * a.FW : (size_t)a.M) * a.OC);
      ee[k] = e;
      if constexpr (ACCUM) {
        size_t ae = e;
        bool hv = true;
        if (a.add_sub > 1) {
          hv = (ph % a.add_sub) == 0 && (pw % a.add_sub) == 0;
          const int hh = a.FH / a.add_sub, ww = a.FW / a.add_sub;
          ae = hv ? (((size_t)nimg * hh + ph / a.add_sub) * ww + pw / a.add_sub) * a.OC + n0 + ccol * 8 : 0;
        }
        has_add[k] = hv;
        va[k] = *reinterpret_cast<const u32x4*>((a.addsrc ? a.addsrc : a.y) + ae);
      }
      if constexpr (EPI > 0) {
        vy[k] = *reinterpret_cast<const u32x4*>(a.ybn + e);
        if constexpr (EPI == 1) vm[k] = a.mbits[e >> 3];
        vy2[k] = *reinterpret_cast<const u32x4*>((has2 ? a.ybn2 : a.ybn) + e);
      }
    }
#pragma unroll
    for (int k = 0; k < G; ++k) {
      u32x4 v = vv[k];
      if constexpr (ACCUM || EPI > 0) {
        float f[8];
        unpack8(v, f);
        if constexpr (ACCUM) {
          float g[8];
          unpack8(va[k], g);
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] += has_add[k] ? g[j] : 0.f;
        }
        if constexpr (EPI > 0) {
          float yv[8];
          unpack8(vy[k], yv);
          if constexpr (EPI == 1) {
#pragma unroll
            for (int j = 0; j < 8; ++j) f[j] = ((vm[k] >> j) & 1u) ? f[j] : 0.f;
          } else {
            float t[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              t[j] = yv[j] * e_sc[j >> 2][j & 3] + e_sh[j >> 2][j & 3];
              f[j] = t[j] > 0.f ? f[j] : 0.f;
            }
            va2[k] = relu_bf16x8(pack8(t));  // the BN output itself (a.a_out write-back)
          }
          v = pack8(f);
          // raw moments of the values actually stored (bf16-rounded): sum g, sum g*y (and g*y2);
          // the centring/scaling by (mean, invstd) is applied once per channel after the
          // reduction: sum g*xhat = inv * (sum g*y - mean * sum g). Rows past M contribute nothing.
          const u32x4 vs = (tail && !ok[k]) ? zero4 : v;
#pragma unroll
          for (int h = 0; h < 4; ++h) {
            const f32x2 gr = {__uint_as_float(vs[h] << 16), __uint_as_float(vs[h] & 0xFFFF0000u)};
            const f32x2 yr = {__uint_as_float(vy[k][h] << 16), __uint_as_float(vy[k][h] & 0xFFFF0000u)};
            ps2[h] += gr;
            pq2[h] = __builtin_elementwise_fma(gr, yr, pq2[h]);
            if (has2) {
              const f32x2 zr = {__uint_as_float(vy2[k][h] << 16), __uint_as_float(vy2[k][h] & 0xFFFF0000u)};
              pr2[h] = __builtin_elementwise_fma(gr, zr, pr2[h]);
            }
          }
        } else {
          v = pack8(f);
        }
      }
      vv[k] = v;
    }
#pragma unroll
    for (int k = 0; k < G; ++k)
      if (ok[k]) *reinterpret_cast<u32x4*>(a.y + ee[k]) = vv[k];
    if constexpr (EPI == 2) {
      if (a.a_out) {  // wave-uniform
#pragma unroll
        for (int k = 0; k < G; ++k)
          if (ok[k]) *reinterpret_cast<u32x4*>(a.a_out + ee[k]) = va2[k];
      }
    }
  };
#pragma unroll
  for (int g0 = 0; g0 + EG <= NIT; g0 += EG) group(g0, std::integral_constant<int, EG>{});
  if constexpr (NIT % EG != 0) group(NIT - NIT % EG, std::integral_constant<int, NIT % EG>{});
  if constexpr (STATS) {
    // per-channel sum / sum of squares of the stored (bf16) tile on the matrix cores instead of the
    // VALU (the statistics were 8-31 % of the expanding 1x1 forwards: profiles/r2s4_probes/): for a
    // 16-channel column group, F = the [32 pixels][16 channels] block of sC read transposed;
    // mfma(ones, F) accumulates the column sums, mfma(F, F) the 16x16 Gram block whose diagonal is
    // the sums of squares. bf16 x bf16 products are exact in fp32. Rows past M are zero (their
    // operands were zero-filled). One fp64 atomic pair per channel into shard tm % nshard.
    constexpr int NCG = BN / 16;
    const int gq = lane >> 4, qq = (lane & 15) >> 2, pq = lane & 3;
    const bf16x8 ones = __builtin_bit_cast(bf16x8, u32x4{0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u});
    double* st = a.stats + (size_t)(tm % a.nshard) * 2 * a.OC;
    for (int cg = wid; cg < NCG; cg += NW) {  // wave-uniform (the transposed reads need full EXEC)
      f32x4 dsum = {0.f, 0.f, 0.f, 0.f}, dsq = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int rb = 0; rb < BM; rb += 32) {
        const int row = rb + 8 * gq + qq;
        const int col = cg * 16 + 4 * pq;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((DBX_LDS s16x4*)(sC + row * (BN + 8) + col));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((DBX_LDS s16x4*)(sC + (row + 4) * (BN + 8) + col));
        const bf16x8 f = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
        dsum = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, f, dsum, 0, 0, 0);
        dsq = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f, f, dsq, 0, 0, 0);
      }
      // D[i][j] sits in lane (i / 4) * 16 + j, register i % 4: column sums in every row (lanes 0-15
      // flush row 0), the diagonal D[j][j] in lane (j / 4) * 16 + j, register j % 4
      const int c = n0 + cg * 16 + (lane & 15);
      if (lane < 16) atomicAdd(st + c, (double)dsum[0]);
      const int dr = (lane & 15) - 4 * gq;
      if (dr >= 0 && dr < 4) {
        const float q = dr == 0 ? dsq[0] : dr == 1 ? dsq[1] : dr == 2 ? dsq[2] : dsq[3];
        atomicAdd(st + a.OC + c, (double)q);
      }
    }
    __syncthreads();  // the LDS is free for reuse when the epilogue returns
  }
  if constexpr (EPI > 0) {
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      bs[2 * h] = ps2[h].x; bs[2 * h + 1] = ps2[h].y;
      bq1[2 * h] = pq2[h].x; bq1[2 * h + 1] = pq2[h].y;
      bq2[2 * h] = pr2[h].x; bq2[2 * h + 1] = pr2[h].y;
    }
    // reduce the per-thread partials over threads with the same chunk column: in-wave lanes
    // l, l+CPR, ... by xor-shuffles, then the 4 waves through LDS, then one atomic per channel
#pragma unroll
    for (int j = 0; j < 8; ++j) {
#pragma unroll
      for (int o = CPR; o < 64; o <<= 1) {
        bs[j] += __shfl_xor(bs[j], o, 64);
        bq1[j] += __shfl_xor(bq1[j], o, 64);
        bq2[j] += __shfl_xor(bq2[j], o, 64);
      }
    }
    __syncthreads();  // sC / sStat reuse
    float* red = reinterpret_cast<float*>(lds);  // [NW waves][3][BN]
    if (lane < CPR) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        red[(wid * 3 + 0) * BN + ccol * 8 + j] = bs[j];
        red[(wid * 3 + 1) * BN + ccol * 8 + j] = bq1[j];
        red[(wid * 3 + 2) * BN + ccol * 8 + j] = bq2[j];
      }
    }
    __syncthreads();
    if (tid < BN) {
      float s = 0.f, q1 = 0.f, q2 = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        s += red[(w * 3 + 0) * BN + tid]; q1 += red[(w * 3 + 1) * BN + tid]; q2 += red[(w * 3 + 2) * BN + tid];
      }
      const int c = n0 + tid;  // raw moments -> sum g*xhat
      q1 = a.inv1[c] * (q1 - a.mean1[c] * s);
      if (has2) q2 = a.inv2[c] * (q2 - a.mean2[c] * s);
      const int shard = (shard % a.nshard);
      double* st1 = a.bstats1 + (size_t)shard * 2 * a.OC;
      atomicAdd(st1 + n0 + tid, (double)s);
      atomicAdd(st1 + a.OC + n0 + tid, (double)q1);
      if (a.bstats2) {
        double* st2 = a.bstats2 + (size_t)shard * 2 * a.OC;
        atomicAdd(st2 + n0 + tid, (double)s);
        atomicAdd(st2 + a.OC + n0 + tid, (double)q2);
      }
    }
  }
  if constexpr (STATS || EPI > 0) {
    if (a.fin1) bn_fin_tail<BM, BN>(a, n0, lds);  // wave-uniform
  }
}

// Split-K combine (IGemmArgs ksplit > 1): every slice stores its fp32 accumulators write-through (sc1)
// to its slab, drains them, and takes a ticket from the tile's counter; the workgroup that draws the
// last ticket reads every slab with sc1 loads (L1 bypassed: the other slices ran on other CUs) and sums
// them in slice order -- bit-identical whichever slice finished last -- then resets the counter for the
// next launch (cdna_hip_programming.md section 5, in-launch split-K reduction; the weight gradient's
// wgrad_store in conv_igemm.hip is the same hand-off). Returns true in the reducer (acc = the sum);
// the LDS is free again when it returns.
template <int TM, int TN, int NT>
__device__ __forceinline__ bool splitk_combine(const IGemmArgs& a, f32x4 (&acc)[TM][TN], const int tile,
                                               const int slice, const int ntile, bf16* lds) {
  constexpr int TILE = TM * TN * NT * 4;  // fp32 elements per tile slab
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const rsrc_t ws = make_rsrc(a.skws, (unsigned long long)a.ksplit * ntile * TILE * 4);
  auto slot = [&](int s, int i, int j) __attribute__((always_inline)) {
    return (unsigned)((((size_t)s * ntile + tile) * TILE + ((size_t)(wid * TM + i) * TN + j) * 256 + lane * 4) * 4);
  };
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), ws, slot(slice, i, j), 0, 16);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's slab has reached memory
  __syncthreads();                                   // ... every wave's; the LDS is no longer read
  int* flag = reinterpret_cast<int*>(lds);
  if (tid == 0) {
    const unsigned t = __hip_atomic_fetch_add((gu32*)(a.skcnt + tile), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    flag[0] = t == (unsigned)(a.ksplit - 1);
  }
  __syncthreads();
  const bool last = flag[0] != 0;
  __syncthreads();  // every wave has read the flag before the epilogue reuses the LDS
  if (!last) return false;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
      acc[i][j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(ws, slot(0, i, j), 0, 16));
  for (int s = 1; s < a.ksplit; ++s) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[i][j] += __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(ws, slot(s, i, j), 0, 16));
  }
  if (tid == 0) __hip_atomic_store((gu32*)(a.skcnt + tile), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}

// TAIL (with PRO), A = x*s + h + (res*rs + rh) computed while staging; the first N tile writes A
// back (tail_out). FWD: the previous residual block's output relu(bn3(x) + shortcut) -- no separate
// bn_apply pass, no re-read of the block output, ReLU mask written too. DGRAD (1x1 stride-1): the
// BN-backward apply dy = k1*g + k2*y + k3 (x = g, res = y, no ReLU) -- the BN-backward apply pass
// is gone and its output is still stored for the weight gradient.
//
// DMA (operand path): 0 = both operands register-staged (two register sets, two LDS buffers);
// 1 = B (weights) moved by LDS-DMA (common.h lds_dma16: no VGPR staging, no ds_write), A register
// staged (it carries the BN prologue); 2 / 3 = both operands by LDS-DMA, a 2- / 3-slot ring (no
// prologue). A DMA wave-instruction fills 8 tile rows x 128 B; the XOR swizzle moves to the
// source side (LDS position (row, slot) receives chunk slot ^ ((row >> 1) & 7) of that row), so
// the fragment reads are unchanged. The ring variants (DMA >= 2) run one tile per workgroup; DMA 1
// (weights only) is persistent like the register-staged path.
// DMA 4: both operands by LDS-DMA in 32-channel stages through a 4-slot ring -- the LDS of the
// 2-slot 64-channel ring (two workgroups per CU stay resident) with three stages instead of one in
// flight behind the MFMAs of the current stage.
template <int BM, int BN, int WM, int WN, int MODE, bool PRO, bool STATS, bool ACCUM, int EPI, bool TAIL = false,
          int DMA = 0>
__global__ __launch_bounds__(64 * WM * WN, 2) void igemm_kernel(const IGemmArgs a) {
  static_assert(DMA == 0 || (MODE != STEM && (DMA == 1 || (!PRO && !TAIL))), "DMA operand path");
  constexpr int NT = 64 * WM * WN;        // threads; WM x WN waves, each owns a (BM/WM) x (BN/WN) tile
  constexpr int NW = WM * WN;
  constexpr int BK = DMA == 4 ? 32 : 64;  // channels per K block (stage)
  constexpr int CPR = BK / 8;             // 16-B chunks per tile row
  constexpr int RPP = NT / CPR;           // tile rows covered per staging pass
  constexpr int A_CH = BM * BK / 8 / NT;  // 16-byte chunks per thread (A)
  constexpr int B_CH = BN * BK / 8 / NT;
  constexpr int TM = BM / (16 * WM), TN = BN / (16 * WN);  // 16x16 MFMA tiles per wave
  constexpr int NBUF = DMA == 3 ? 3 : DMA == 4 ? 4 : 2;  // LDS operand buffers (ring slots)
  constexpr int LDS_AB = NBUF * (BM + BN) * BK;  // bf16 elements
  constexpr int LDS_C = BM * (BN + 8);
  constexpr int LDS_RED = 2 * (3 * NW * BN);  // fp32 reduction scratch (in bf16 units)
  constexpr int PRO_MAXC = TAIL ? 1024 : 512;              // prologue channels held in LDS (host-checked)
  constexpr int LDS_PRO = (PRO && MODE != STEM) ? (TAIL ? 8 : 4) * PRO_MAXC : 0;  // fp32 arrays (bf16 units)
  constexpr int LDS_MAIN = (LDS_AB > LDS_C + LDS_RED) ? LDS_AB : (LDS_C + LDS_RED);
  __shared__ __attribute__((aligned(16))) bf16 lds[LDS_MAIN + LDS_PRO];
  bf16* sA = lds;                  // [NBUF][BM][BK]
  bf16* sB = lds + NBUF * BM * BK; // [NBUF][BN][BK]
  // prologue affine of ALL input channels, staged once: the per-block coefficients are read from
  // LDS at transform time instead of living in registers across the pipeline
  float* sPro = reinterpret_cast<float*>(lds + LDS_MAIN);  // [2 or 4][PRO_MAXC]: scale, shift (, rs, rh)

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wm = wid / WN, wn = wid % WN;
  const int ntn = a.OC / BN, ntm = (a.M + BM - 1) / BM, ntile = ntn * ntm;
  // Persistent tiles: workgroup b computes tiles b, b + G, b + 2G, ... (G = gridDim.x, a multiple
  // of 8 sized by the host to the resident capacity, so tile t stays on XCD t % 8 and xcd_remap
  // still groups A-sharing tiles per L2). The next tile's first K block is loaded while this
  // tile's epilogue runs: short-K (1x1) convs no longer leave the CU idle during load latency.
  // The "l" indices are the LOADER's tile (the one being staged), m0/n0/tm the epilogue's.
  int ltm = 0, ltn = 0, lm0 = 0, ln0 = 0;
  int lk = 0, lcb = 0, lts = 0, ltr = 0;  // next K block to load (see advance())
  const int KTOT = (MODE == STEM) ? 256 : a.R * a.S * a.IC;  // weight row length
  const int cpt = (MODE == STEM) ? 1 : a.IC / BK;              // K blocks per tap
  const int KB = (MODE == STEM) ? 4 : a.nr * a.ns * cpt;
  // split-K (a.ksplit > 1; register-staged A operand paths only, never STEM, never persistent): this
  // workgroup's tile, slice and K-block range (the LDS-DMA ring variants compile without it: +15-60 VGPRs)
  const bool split = MODE != STEM && DMA <= 1 && a.ksplit > 1;  // workgroup-uniform
  int ltile = 0, slice = 0, kb_lo = 0, kb_hi = KB;

  // ---- per-thread A rows: decompose output pixel once per tile ---------------------
  const int ach = tid & (CPR - 1);
  // LDS-DMA: the chunk this lane fetches for each of its rows (row = tid/CPR + RPP*i: RPP is a
  // multiple of 16, so the swizzle term is the same for all i)
  const int lch = ach ^ fswz<BK>(tid / CPR);
  const int acha = DMA >= 2 ? lch : ach;  // A chunk loaded by this thread
  const bf16* abase[A_CH];   // STEM mode: image base
  int ahb[A_CH], awb[A_CH];  // top-left input coordinate of the row's receptive field
  unsigned apix[A_CH];       // byte offset of (n, ahb, awb, ach*8) in x (host: bytes < kOOB)
  auto set_tile = [&](int t) __attribute__((always_inline)) {
    int bid;
    if (split) {  // a tile's slices are consecutive remapped ids: one XCD's L2 holds its slabs
      const int id = xcd_remap(t, ntile * a.ksplit);
      bid = id / a.ksplit;
      slice = id - bid * a.ksplit;
      kb_lo = slice * a.kper;
      kb_hi = kb_lo + a.kper < KB ? kb_lo + a.kper : KB;
    } else {
      bid = xcd_remap(t, ntile);
    }
    ltile = bid;
    ltm = bid / ntn; ltn = bid - ltm * ntn;
    lm0 = ltm * BM; ln0 = ltn * BN;
    lk = kb_lo;
    lcb = kb_lo % cpt;
    lts = (kb_lo / cpt) % a.ns;
    ltr = (kb_lo / cpt) / a.ns;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int m = lm0 + tid / CPR + RPP * i;
      const int ohw = a.OH * a.OW;
      int n = mdiv_or(m, a.mag_ohw, ohw);
      const int pq = m - n * ohw;
      const int oh = mdiv_or(pq, a.mag_ow, a.OW), ow = pq - oh * a.OW;
      if (m >= a.M) { n = 0; }
      abase[i] = a.x + (size_t)n * a.IH * a.IW * a.IC;
      if (MODE == DGRAD) { ahb[i] = oh + a.dh0; awb[i] = ow + a.dw0; }
      else { ahb[i] = oh * a.stride - a.pad; awb[i] = ow * a.stride - a.pad; }
      apix[i] = 2u * (unsigned)(((n * a.IH + ahb[i]) * a.IW + awb[i]) * a.IC + acha * 8);
      // a live row's sample lies inside x (its taps then add in-image displacements only)
      DBX_DCHECK(m >= a.M || (n >= 0 && n < a.N && oh >= 0 && oh < a.OH && ow >= 0 && ow < a.OW));
      if (m >= a.M) ahb[i] = -(1 << 28);
    }
  };
  int tcur = blockIdx.x;
  set_tile(tcur);
  const rsrc_t xr = make_rsrc(a.x, 2ull * a.N * a.IH * a.IW * a.IC);
  const rsrc_t wr = make_rsrc(a.w, 2ull * a.OC * KTOT);
  const int NKB = kb_hi - kb_lo;  // K blocks of this workgroup (all of them unless split)

  // Two register staging sets: the loads of block kb+2 are issued while block kb+1's data (set
  // issued one iteration earlier) is still landing, so each global load has two blocks of MFMA
  // work to hide its latency instead of one. The K loop is unrolled by two so S is a constant.
  u32x4 ra[2][A_CH], rb[2][B_CH];
  u32x4 rr[2][TAIL ? A_CH : 1];           // TAIL: staged shortcut chunks
  const u32x4 zero4 = {0u, 0u, 0u, 0u};
  unsigned avalid[2] = {0u, 0u};          // bit i: chunk i is a real (non-padding) tap
  int pcb[2] = {0, 0};                    // channel block of the staged set (prologue coefficients)
  if constexpr (PRO && MODE != STEM) {
    for (int c = tid; c < a.IC; c += NT) {
      if (a.fin_in) {  // wave-uniform: the input BN finalized here (workgroup 0 stores it)
        float sc, sh;
        bn_fin_consume(a.fin_in[0], c, blockIdx.x == 0, sc, sh);
        sPro[c] = sc;
        sPro[PRO_MAXC + c] = sh;
        if constexpr (TAIL) {  // forward tail: fin_in[1] is the shortcut's BN when it has one
          float rs = 1.f, rh = 0.f;
          if (a.res_scale) bn_fin_consume(a.fin_in[1], c, blockIdx.x == 0, rs, rh);
          sPro[2 * PRO_MAXC + c] = rs;
          sPro[3 * PRO_MAXC + c] = rh;
        }
        continue;
      }
      sPro[c] = a.in_scale[c];
      sPro[PRO_MAXC + c] = a.in_shift[c];
      if constexpr (TAIL) {
        sPro[2 * PRO_MAXC + c] = a.res_scale ? a.res_scale[c] : 1.f;
        sPro[3 * PRO_MAXC + c] = a.res_shift ? a.res_shift[c] : 0.f;
      }
    }
    __syncthreads();
  }
  // TAIL write-back: wave-uniform per staged set (first N tile, live block)
  bool wlive[2] = {false, false};
  unsigned wtoff[2] = {0u, 0u};
  const rsrc_t rresr = make_rsrc(a.res, TAIL ? 2ull * a.N * a.IH * a.IW * a.IC : 0ull);
  const rsrc_t toutr = make_rsrc(a.tail_out, (TAIL && a.tail_out) ? 2ull * a.N * a.IH * a.IW * a.IC : 0ull);
  const rsrc_t tbitr = make_rsrc(a.tail_bits, (TAIL && a.tail_bits) ? 1ull * a.N * a.IH * a.IW * a.IC / 8 : 0ull);
  // decomposition of the NEXT block to load (kb -> channel block, tap row, tap column), advanced
  // by one per load instead of dividing kb (wave-uniform scalars). The pipeline's unconditional
  // prefetch runs two blocks past the end: those loads use an out-of-range offset for every lane,
  // so they cost an instruction issue but no memory traffic (short-K 1x1 convs: KB = 1..4)
  auto advance = [&]() __attribute__((always_inline)) {
    ++lk;
    if (++lcb == cpt) { lcb = 0; if (++lts == a.ns) { lts = 0; ++ltr; } }
  };

  auto load_a = [&](int S) __attribute__((always_inline)) {
    if constexpr (MODE == STEM) {
      // k block lk covers filter rows r = 2lk, 2lk+1; chunk ach: r = 2lk + (ach>>2), pixels
      // s = 2*(ach&3), +1, 4 channels (8 bytes) each.
      const int r = 2 * (lk < KB ? lk : KB - 1) + (ach >> 2);
      const int s0 = 2 * (ach & 3);
#pragma unroll
      for (int i = 0; i < A_CH; ++i) {
        const int ih = ahb[i] + r;
        const bool rv = (r < a.R) && ih >= 0 && ih < a.IH;
        unsigned int w4[4];
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          // branch-free: an out-of-image pixel loads the image base and is zeroed by the select
          const int s = s0 + p, iw = awb[i] + s;
          const bool v = rv && s < a.S && (unsigned)iw < (unsigned)a.IW;
          const uint2 t = *reinterpret_cast<const uint2*>(abase[i] + (v ? (ih * a.IW + iw) * 4 : 0));
          w4[2 * p] = v ? t.x : 0u; w4[2 * p + 1] = v ? t.y : 0u;
        }
        ra[S][i] = u32x4{w4[0], w4[1], w4[2], w4[3]};
      }
    } else {
      const int cb = lcb * BK;
      const int r = a.r0 + a.tstep * ltr, s = a.s0 + a.tstep * lts;
      if constexpr (PRO) pcb[S] = cb;
      if constexpr (TAIL) { wlive[S] = lk < kb_hi && ltn == 0; wtoff[S] = 2u * (unsigned)cb; }
      // tap displacement, the same for all of this thread's rows (uniform, bytes)
      const int dh = (MODE == DGRAD) ? -ltr : r, dw = (MODE == DGRAD) ? -lts : s;
      const unsigned toff = 2u * (unsigned)((dh * a.IW + dw) * a.IC + cb);
      const bool live = lk < kb_hi;  // wave-uniform: false for the prefetches past the last block
      avalid[S] = 0;
#pragma unroll
      for (int i = 0; i < A_CH; ++i) {
        const bool v = live && (unsigned)(ahb[i] + dh) < (unsigned)a.IH && (unsigned)(awb[i] + dw) < (unsigned)a.IW;
        // padding taps / rows past M read out of the buffer's range: the hardware returns zeros
        DBX_DCHECK(!v || (unsigned long long)(apix[i] + toff) + 16ull <= 2ull * a.N * a.IH * a.IW * a.IC);
        ra[S][i] = buf_load16(xr, v ? apix[i] + toff : kOOB);
        if constexpr (TAIL) rr[S][i] = buf_load16(rresr, v ? apix[i] + toff : kOOB);
        if constexpr (PRO) avalid[S] |= (v ? 1u : 0u) << i;
      }
    }
  };
  // BN-apply (+ReLU) prologue on the staged A chunks. Kept apart from load_a so the global loads
  // of block kb+1 stay in flight across block kb's MFMAs (the transform waits on the data).
  auto pro_a = [&](int S) __attribute__((always_inline)) {
    if constexpr (TAIL && MODE != STEM) {
      // TAIL: four affine vectors per channel; transformed one 4-channel half at a time, in place
      // (the half's result replaces the half's raw dwords), so 16 instead of 32 coefficient
      // registers are live next to the two staged sets: the 128 x 128 / 256 x 128 tail variants
      // spilled inside the K loop with all eight vectors resident
      const int c0 = pcb[S] + ach * 8;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f32x4 ps = *reinterpret_cast<const f32x4*>(sPro + c0 + 4 * h);
        const f32x4 ph = *reinterpret_cast<const f32x4*>(sPro + PRO_MAXC + c0 + 4 * h);
        const f32x4 pr = *reinterpret_cast<const f32x4*>(sPro + 2 * PRO_MAXC + c0 + 4 * h);
        const f32x4 pq = *reinterpret_cast<const f32x4*>(sPro + 3 * PRO_MAXC + c0 + 4 * h);
#pragma unroll
        for (int i = 0; i < A_CH; ++i) {
          float f[4], g[4];
#pragma unroll
          for (int d = 0; d < 2; ++d) {
            const unsigned xv = ra[S][i][2 * h + d], rv = rr[S][i][2 * h + d];
            f[2 * d] = __uint_as_float(xv << 16); f[2 * d + 1] = __uint_as_float(xv & 0xFFFF0000u);
            g[2 * d] = __uint_as_float(rv << 16); g[2 * d + 1] = __uint_as_float(rv & 0xFFFF0000u);
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            f[j] = f[j] * ps[j] + ph[j];
            f[j] += g[j] * pr[j] + pq[j];  // + shortcut (identity: rs = 1, rh = 0), as bn_apply computes it
          }
          ra[S][i][2 * h] = pack2(f[0], f[1]);
          ra[S][i][2 * h + 1] = pack2(f[2], f[3]);
        }
      }
#pragma unroll
      for (int i = 0; i < A_CH; ++i) {
        u32x4 t = ra[S][i];
        if constexpr (MODE != DGRAD) t = relu_bf16x8(t);  // forward PRO implies ReLU (host-checked)
        const bool vi = (avalid[S] >> i) & 1u;
        ra[S][i] = vi ? t : zero4;  // padding taps stay exactly zero
        // block output + 1-bit mask (bit j: element j > 0) written back by the first N tile
        const unsigned off = (wlive[S] && vi) ? apix[i] + wtoff[S] : kOOB;
        buf_store16(toutr, off, t);
        if constexpr (MODE == DGRAD) continue;
        unsigned bits = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q)
          bits |= (((t[q] & 0xFFFFu) ? 1u : 0u) << (2 * q)) | (((t[q] >> 16) ? 1u : 0u) << (2 * q + 1));
        buf_store8(tbitr, off == kOOB ? kOOB : (off >> 4), (unsigned char)bits);
      }
    } else if constexpr (PRO && MODE != STEM) {
      const int c0 = pcb[S] + ach * 8;  // this thread's 8 channels (the same for all its rows)
      const f32x4 ps0 = *reinterpret_cast<const f32x4*>(sPro + c0);
      const f32x4 ps1 = *reinterpret_cast<const f32x4*>(sPro + c0 + 4);
      const f32x4 ph0 = *reinterpret_cast<const f32x4*>(sPro + PRO_MAXC + c0);
      const f32x4 ph1 = *reinterpret_cast<const f32x4*>(sPro + PRO_MAXC + c0 + 4);
      f32x4 pr0, pr1, pq0, pq1;
      if constexpr (TAIL) {
        pr0 = *reinterpret_cast<const f32x4*>(sPro + 2 * PRO_MAXC + c0);
        pr1 = *reinterpret_cast<const f32x4*>(sPro + 2 * PRO_MAXC + c0 + 4);
        pq0 = *reinterpret_cast<const f32x4*>(sPro + 3 * PRO_MAXC + c0);
        pq1 = *reinterpret_cast<const f32x4*>(sPro + 3 * PRO_MAXC + c0 + 4);
      }
#pragma unroll
      for (int i = 0; i < A_CH; ++i) {
        float f[8];
        unpack8(ra[S][i], f);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          f[j] = f[j] * ps0[j] + ph0[j];
          f[j + 4] = f[j + 4] * ps1[j] + ph1[j];
        }
        if constexpr (TAIL) {  // + shortcut (identity: rs = 1, rh = 0), as bn_apply computes it
          float g[8];
          unpack8(rr[S][i], g);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            f[j] += g[j] * pr0[j] + pq0[j];
            f[j + 4] += g[j + 4] * pr1[j] + pq1[j];
          }
        }
        u32x4 t = pack8(f);
        if constexpr (MODE != DGRAD) t = relu_bf16x8(t);  // forward PRO implies ReLU (host-checked)
        const bool vi = (avalid[S] >> i) & 1u;
        ra[S][i] = vi ? t : zero4;  // padding taps stay exactly zero
        if constexpr (TAIL) {
          // block output + 1-bit mask (bit j: element j > 0) written back by the first N tile
          const unsigned off = (wlive[S] && vi) ? apix[i] + wtoff[S] : kOOB;
          buf_store16(toutr, off, t);
          if constexpr (MODE == DGRAD) continue;
          unsigned bits = 0;
#pragma unroll
          for (int q = 0; q < 4; ++q)
            bits |= (((t[q] & 0xFFFFu) ? 1u : 0u) << (2 * q)) | (((t[q] >> 16) ? 1u : 0u) << (2 * q + 1));
          buf_store8(tbitr, off == kOOB ? kOOB : (off >> 4), (unsigned char)bits);
        }
      }
    }
  };
  auto load_b = [&](int S) __attribute__((always_inline)) {
    int koff;
    if constexpr (MODE == STEM) {
      koff = lk * BK + ach * 8;
    } else {
      koff = ((a.r0 + a.tstep * ltr) * a.S + a.s0 + a.tstep * lts) * a.IC + lcb * BK + ach * 8;
    }
    const bool live = lk < kb_hi;
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int n = ln0 + tid / CPR + RPP * i;
      DBX_DCHECK(!live || (n < a.OC && koff + 8 <= KTOT));
      rb[S][i] = buf_load16(wr, live ? 2u * (unsigned)(n * KTOT + koff) : kOOB);
    }
  };
  auto store_a = [&](int buf, int S) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int row = tid / CPR + RPP * i;
      *reinterpret_cast<u32x4*>(sA + buf * BM * BK + row * BK + ((ach ^ fswz<BK>(row)) << 3)) = ra[S][i];
    }
  };
  auto store_ab = [&](int buf, int S) __attribute__((always_inline)) {
    store_a(buf, S);
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int row = tid / CPR + RPP * i;
      *reinterpret_cast<u32x4*>(sB + buf * BN * BK + row * BK + ((ach ^ fswz<BK>(row)) << 3)) = rb[S][i];
    }
  };
  // ---- LDS-DMA operand path (DMA > 0) ----
  // wave wid's DMA instruction i fills tile rows RPP*i + 8*wid .. +7 (1 KiB) of the slot's image
  const unsigned lds0 = lds_addr(lds);
  const i32x4 xsrd = make_srd(a.x, (MODE == STEM || DMA < 2) ? 0ull : 2ull * a.N * a.IH * a.IW * a.IC);
  const i32x4 wsrd = make_srd(a.w, DMA == 0 ? 0ull : 2ull * a.OC * KTOT);
  // B: the DMA-ed weights run ahead of A by one block less than the register pipeline (DMA 1), so
  // they keep their own K-block position (bk: block, bcb / bts / btr: channel block, tap column, row)
  int bk = kb_lo, bcb = kb_lo % cpt, bts = (kb_lo / cpt) % a.ns, btr = (kb_lo / cpt) / a.ns;
  auto dma_b = [&](int buf) __attribute__((always_inline)) {
    const int koff = ((a.r0 + a.tstep * btr) * a.S + a.s0 + a.tstep * bts) * a.IC + bcb * BK + lch * 8;
    const bool live = bk < kb_hi;  // past the last block: out-of-range offsets (zeros, no traffic)
    const unsigned dst = lds0 + 2u * (unsigned)(NBUF * BM * BK + buf * BN * BK) + 1024u * (unsigned)wid;
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int n = ln0 + tid / CPR + RPP * i;
      lds_dma16(wsrd, live ? 2u * (unsigned)(n * KTOT + koff) : kOOB, dst + 1024u * (unsigned)(NW * i));
    }
    ++bk;
    if (++bcb == cpt) { bcb = 0; if (++bts == a.ns) { bts = 0; ++btr; } }
  };
  // A (DMA >= 2, no prologue): the gather of load_a for the block at the loader position
  auto dma_a = [&](int buf) __attribute__((always_inline)) {
    const int cb = lcb * BK;
    const int r = a.r0 + a.tstep * ltr, s = a.s0 + a.tstep * lts;
    const int dh = (MODE == DGRAD) ? -ltr : r, dw = (MODE == DGRAD) ? -lts : s;
    const unsigned toff = 2u * (unsigned)((dh * a.IW + dw) * a.IC + cb);
    const bool live = lk < kb_hi;
    const unsigned dst = lds0 + 2u * (unsigned)(buf * BM * BK) + 1024u * (unsigned)wid;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const bool v = live && (unsigned)(ahb[i] + dh) < (unsigned)a.IH && (unsigned)(awb[i] + dw) < (unsigned)a.IW;
      lds_dma16(xsrd, v ? apix[i] + toff : kOOB, dst + 1024u * (unsigned)(NW * i));
    }
  };

  f32x4 acc[TM][TN];

  auto mma = [&](int buf) __attribute__((always_inline)) {
    const bf16* cA = sA + buf * BM * BK;
    const bf16* cB = sB + buf * BN * BK;
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      bf16x8 af[TM], bfr[TN];
      const int ch = ks * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * (BM / WM) + i * 16 + (lane & 15);
        af[i] = *reinterpret_cast<const bf16x8*>(cA + row * BK + ((ch ^ fswz<BK>(row)) << 3));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * (BN / WN) + j * 16 + (lane & 15);
        bfr[j] = *reinterpret_cast<const bf16x8*>(cB + row * BK + ((ch ^ fswz<BK>(row)) << 3));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          // operands swapped (C^T = W X^T): a lane's 4 accumulators are 4 consecutive output
          // channels of one pixel, so the epilogue stages them with one 8-byte LDS write
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    }
  };
  // one pipeline step on block kb (LDS buffer kb&1, register set S holds block kb+1)
  // The prefetch is issued unconditionally (past the end it re-reads the last block, data unused)
  // and the loop body is branch-free, so hipcc's waitcnt pass sees the same in-flight loads on
  // every path and waits only for the older set (counted vmcnt) instead of draining to vmcnt(0).
  auto step = [&](int kb, int S) __attribute__((always_inline)) {
    load_a(S ^ 1);  // block kb + 2 (past the slice's end: no traffic)
    load_b(S ^ 1);
    advance();
    mma(kb & 1);
    pro_a(S);
    store_ab((kb + 1) & 1, S);  // past the last block this fills the idle buffer, never read
    __syncthreads();
  };

  if constexpr (DMA == 0) {
    load_a(0);
    load_b(0);
    advance();
  } else if constexpr (DMA == 1) {
    load_a(0);  // (B by DMA at the top of the tile loop)
    advance();
  }
  for (;;) {  // persistent tile loop (exit: every wave of the workgroup leaves after the same tile)
  if constexpr (DMA == 0) {
  load_a(1);
  load_b(1);
  advance();
  pro_a(0);
  store_ab(0, 0);
  __syncthreads();
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  int kb = 0;
  for (; kb + 1 < NKB; kb += 2) {
    step(kb, 1);
    step(kb + 1, 0);
  }
  if (kb < NKB) {
    mma(kb & 1);
    __syncthreads();  // the epilogue's sC staging aliases the operand buffers
  }
  } else if constexpr (DMA == 1) {
    // B by LDS-DMA one block ahead, A register-staged two blocks ahead (its BN prologue runs
    // after the MFMAs of the current block). The vector-memory ops a wave has in flight at the
    // end of step kb, oldest first: B(kb+1) DMA, A(kb+2) loads, the tail write-back stores of
    // A(kb+1): the counted wait retires B(kb+1) and leaves the rest in flight.
    // (A(0) is already in flight: issued before the loop, or before the previous tile's epilogue)
    // TAIL: load_a issues two loads per chunk (x and the shortcut / BN operand), pro_a one (DGRAD:
    // tail_out) or two (FWD: + mask bits) stores; the counted wait must leave exactly the A(kb+2)
    // loads and the stores in flight -- one chunk's worth fewer would also retire half of A(kb+2)
    constexpr int A_LD = TAIL ? 2 * A_CH : A_CH;
    constexpr int TAIL_ST = TAIL ? (MODE == DGRAD ? A_CH : 2 * A_CH) : 0;
    dma_b(0);
    load_a(1);
    advance();
    pro_a(0);
    store_a(0, 0);
    dma_wait<A_LD + TAIL_ST>();  // A(0), B(0) (older than the A(1) loads and the tail stores)
    __syncthreads();
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto stepd = [&](int kb, int S) __attribute__((always_inline)) {
      dma_b((kb + 1) & 1);  // slot (kb+1)&1 was last read by mma(kb-1): free after the barrier
      load_a(S ^ 1);
      advance();
      mma(kb & 1);
      pro_a(S);
      store_a((kb + 1) & 1, S);
      dma_wait<A_LD + TAIL_ST>();
      __syncthreads();
    };
    int kb = 0;
    for (; kb + 1 < NKB; kb += 2) {
      stepd(kb, 1);
      stepd(kb + 1, 0);
    }
    if (kb < NKB) mma(kb & 1);
    dma_wait<0>();    // no DMA may still write the LDS the epilogue stages through
    __syncthreads();
  } else {
    // both operands by LDS-DMA through an NBUF-slot ring (block kb + NBUF - 1 issued while block
    // kb is computed); past the last block the issues read out of range (zeros into an idle slot)
    constexpr int ND = A_CH + B_CH;  // DMA instructions per wave and block
#pragma unroll
    for (int sl = 0; sl < NBUF - 1; ++sl) {
      dma_a(sl);
      dma_b(sl);
      advance();
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    int cur = 0;
    for (int kb = 0; kb < NKB; ++kb) {
      dma_wait<(NBUF - 2) * ND>();  // this wave's part of block kb has landed
      __syncthreads();              // ... every wave's; and the slot issued next is no longer read
      const int nxt = cur == 0 ? NBUF - 1 : cur - 1;
      dma_a(nxt);
      dma_b(nxt);
      advance();
      mma(cur);
      cur = cur + 1 == NBUF ? 0 : cur + 1;
    }
    dma_wait<0>();
    __syncthreads();
  }
  // this tile's indices for the epilogue; then stage the next tile's first K block (register set
  // 0) so its loads are in flight during the epilogue
  // (PF: plain / forward-stats epilogues; the BN-backward epilogues hold too many registers to
  // keep a staged block alive across them, so those stage the next tile after the epilogue)
  // Only those run persistent (PF); the rest leave the loop after one tile (the host launches
  // one workgroup per tile for them), which compiles to the straight-line single-tile kernel.
  // DMA 1 (weights by LDS-DMA): A(0) of the next tile is staged in registers the same way, its
  // weights are DMA-ed at the top of the next iteration (they land in the LDS the epilogue stages
  // C through, so only after the barrier below)
  constexpr bool PF = EPI == 0 && !ACCUM && !TAIL && !(BM == 256 && BN == 64) && DMA <= 1;  // (+: register room)
  const int m0 = lm0, n0 = ln0, tm = ltm;
  if (split) {  // (workgroup-uniform) the slices' sum in slice order: only the last arriver continues
    if (!splitk_combine<TM, TN, NT>(a, acc, ltile, slice, ntile, lds)) return;
  }
  tcur += gridDim.x;
  const bool more = PF && !split && tcur < ntile;  // workgroup-uniform
  if (more) {  // A (activations, HBM latency) now; B (weights, L2-resident) after the epilogue
    set_tile(tcur);
    load_a(0);
    if constexpr (DMA == 1) {
      advance();
      bk = bcb = bts = btr = 0;  // (persistent launches are never split: the slice is all of K)
    }
  }

  igemm_epilogue<BM, BN, WM, WN, MODE, STATS, ACCUM, EPI>(a, acc, lds, m0, n0, tm, blockIdx.x);
  if (!more) break;
  if constexpr (DMA == 0) {
    load_b(0);
    advance();
  }
  __syncthreads();  // the epilogue's LDS reads are done before the next tile's staging writes
  }
}

}  // namespace dbx

// ---- host launch helper (shared by the conv TUs) --------------------------------------------
namespace dbx {
template <int BM, int BN, int MODE, bool PRO, bool STATS, bool ACCUM, int EPI, bool TAIL = false, int DMA = 0>
static int launch_igemm_t(const IGemmArgs& a, hipStream_t st) {
  // tile shape -> wave layout: 128x128, 128x64, 64x64 on 2x2 waves (256 threads, 2 blocks/CU);
  // 256x128 on 4x2 and 128x256 on 2x4 waves (512 threads, 1 block/CU, 96 KB LDS); 256x64 on 4x1
  // waves (64x64 per wave like 128x128: 2/3 of the LDS bytes per MFMA of 64x32 wave tiles, for
  // the 64-channel layers)
  constexpr int WM = (BM == 256) ? 4 : 2;
  constexpr int WN = (BN == 256) ? 4 : (BM == 256 && BN == 64) ? 1 : 2;
  const int ntile = (a.OC / BN) * ((a.M + BM - 1) / BM);
  // persistent grid: the resident capacity (occupancy x CUs), a multiple of 8 (XCD round-robin)
  static const int cap = [] {
    int per_cu = 0, dev = 0, cus = 0;
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &per_cu, reinterpret_cast<const void*>(&igemm_kernel<BM, BN, WM, WN, MODE, PRO, STATS, ACCUM, EPI, TAIL, DMA>),
        64 * WM * WN, 0);
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (per_cu <= 0 || cus <= 0) return 1 << 30;
    return (per_cu * cus) & ~7;
  }();
  constexpr bool PF = EPI == 0 && !ACCUM && !TAIL && !(BM == 256 && BN == 64) && DMA <= 1;  // persistent (see the kernel)
  // the weights-by-DMA variants walk tiles only when each workgroup gets at least 8 of them: headline
  // ResNet-50 b1024 +0.8 %, the TinyImageNet step (~4 tiles per workgroup) -0.3 % when they always do
  // (profiles/r5_persist_dma1/)
  constexpr int kPersistDma1 = 8;
  const bool one_per_wg = DMA == 1 && ntile < (long long)kPersistDma1 * cap;
  const int nwg = a.ksplit > 1 ? ntile * a.ksplit : (!PF || ntile <= cap || one_per_wg) ? ntile : cap;
  hipLaunchKernelGGL((igemm_kernel<BM, BN, WM, WN, MODE, PRO, STATS, ACCUM, EPI, TAIL, DMA>), dim3(nwg), dim3(64 * WM * WN), 0, st, a);
  return (int)hipGetLastError();
}

// operand-path selection: a prologue (PRO / TAIL) keeps A in registers -> DMA 0 or 1 (B by DMA);
// plain operands -> DMA 0, 2 or 3 (ring depth; a request of 1 means 2)
#define DBX_DMA_PRO(CALL, ...) \
  return dma ? CALL<__VA_ARGS__, 1>(a, st) : CALL<__VA_ARGS__, 0>(a, st)
// (tile code 6 = the 4-slot ring of 32-channel stages, kernel DMA 4)
#define DBX_DMA_PLAIN(CALL, ...)                         \
  return dma == 6 ? CALL<__VA_ARGS__, 4>(a, st)          \
         : dma == 3 ? CALL<__VA_ARGS__, 3>(a, st)        \
         : dma ? CALL<__VA_ARGS__, 2>(a, st) : CALL<__VA_ARGS__, 0>(a, st)

}  // namespace dbx

#define DBX_TILES(F, ...)                                                         \
  if (bm == 128 && bn == 128) return F<128, 128>(__VA_ARGS__);                    \
  if (bm == 128 && bn == 64) return F<128, 64>(__VA_ARGS__);                      \
  if (bm == 64 && bn == 64) return F<64, 64>(__VA_ARGS__);                        \
  if (bm == 256 && bn == 128) return F<256, 128>(__VA_ARGS__);                    \
  if (bm == 128 && bn == 256) return F<128, 256>(__VA_ARGS__);                    \
  if (bm == 256 && bn == 64) return F<256, 64>(__VA_ARGS__);


