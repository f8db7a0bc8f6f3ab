// Fused stem backward: max-pool backward + stem BN-backward apply + stem weight gradient in ONE pass
// (SURVEY.md §2.4 K3/K5/K7/K10 for the ResNet stem; the reference runs MaxPool2d backward, the
// cuDNN BatchNorm backward and the cuDNN conv weight gradient as separate HBM passes).
//
// For every stem output pixel (n, h, w) and channel c:
//   g  = sum over the <= 2 x 2 pooling windows that contain (h, w) and whose argmax it is of dpool
//   g  = [y*sc + sh > 0] * g                      (the ReLU after the stem BN)
//   dy = k1*g + k2*y + k3                         (BN-backward apply, rounded to bf16)
//   dW[c][r][s][ci] += dy * x4[n][h*stride - pad + r][w*stride - pad + s][ci]
// dy lives only in LDS: the unfused schedule wrote it (N x 112 x 112 x 64 bf16 = 1.6 GB at batch 1024)
// and the weight-gradient pass read it back. The weight gradient uses the stem layout of the forward
// kernels: taps padded to 8 x 8 pixels x 4 channels (KT = 256 columns), k-major fp32 slabs.
//
// Split-K over pixels: workgroup s owns pixels [s*m_per_split, ...) in 64-pixel K-blocks, 2x2 waves
// each owning 32 output channels x 128 tap columns; one register set of raw inputs in flight under
// the current block's MFMAs, double-buffered LDS images (tr_swz: conflict-free staging stores and
// transposed fragment reads, as in the wgrad kernels). One fp32 slab per workgroup; wgrad_reduce
// sums the slabs in a fixed order (deterministic).
#include "common.h"
#include "abi.h"

namespace dbx {

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ u32x2 buf_load8(rsrc_t r, unsigned off) {
  return __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
}

// FUSED = false: the plain stem weight gradient from a stored dy (a.y), same tiles / pipeline: one
// 64 x 256 tile per workgroup, so dy is read once (the generic wgrad kernel splits the 256 tap
// columns over two workgroups that each read it).
template <bool FUSED>
__global__ __launch_bounds__(256, 2) void stem_bwd_kernel(const StemBwdArgs a) {
  constexpr int C = 64, KT = 256, BKM = 64;
  constexpr int TM = 2, TN = 8;  // wave (wm, wn): 32 output channels x 128 tap columns
  __shared__ __attribute__((aligned(16))) bf16 lds[2 * BKM * (C + KT)];
  bf16* sA = lds;                // [2][BKM][C]  dy (tr_swz, 8 chunks per row)
  bf16* sB = lds + 2 * BKM * C;  // [2][BKM][KT] im2col(x4) (tr_swz, 32 chunks per row)

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wm = wid >> 1, wn = wid & 1;
  const int split = blockIdx.x;
  const int mbeg = split * a.m_per_split;
  const int mend = min(a.M, mbeg + a.m_per_split);
  const int nkb = (mend - mbeg + BKM - 1) / BKM;
  // dy loader: pixel rows arow + 32 i (i < 2), one 8-channel group ach per thread
  const int arow = tid >> 3, ach = tid & 7;
  // x4 loader: pixel row brow; chunk bc + 4 j holds filter row r = j, tap pixels s = 2 bc, 2 bc + 1
  const int brow = tid >> 2, bc = tid & 3;
  const rsrc_t dpr = make_rsrc(a.dpool, 2ull * a.N * a.P * a.Q * C);
  const rsrc_t agr = make_rsrc(a.arg, 1ull * a.N * a.P * a.Q * C);
  const rsrc_t yr = make_rsrc(a.y, 2ull * a.M * C);
  const rsrc_t xr = make_rsrc(a.x4, 8ull * a.N * a.IH * a.IW);
  const int HW = a.H * a.W;

  // raw inputs of one K-block: per dy row, the 4 candidate windows' pooled gradients / argmax bytes,
  // the window-local index this pixel has in each (packed bytes), and y; per x4 chunk two pixels
  u32x4 rgd[2][4], ry[2];
  u32x2 rav[2][4], rb[8][2];
  unsigned rme[2];
  auto load = [&](int kb) __attribute__((always_inline)) {
    const int m0 = mbeg + kb * BKM;
    const int mlim = kb < nkb ? mend : 0;  // past the last block: every offset out of range (zeros)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int m = m0 + arow + 32 * i;
      const bool mv = m < mlim;
      if constexpr (!FUSED) {
        ry[i] = buf_load16(yr, mv ? 2u * (unsigned)(m * C + ach * 8) : kOOB);
        continue;
      }
      const int n = mdiv(m, a.mag_hw), hw = m - n * HW;
      const int h = mdiv(hw, a.mag_w), w = hw - h * a.W;
      const int p_lo = max(0, (h + a.ppad - a.PK + a.pstride) / a.pstride);
      const int p_hi = min(a.P - 1, (h + a.ppad) / a.pstride);
      const int q_lo = max(0, (w + a.ppad - a.PK + a.pstride) / a.pstride);
      const int q_hi = min(a.Q - 1, (w + a.ppad) / a.pstride);
      unsigned me = 0;
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int p = p_lo + u, q = q_lo + t;
          const int r = h + a.ppad - p * a.pstride, s = w + a.ppad - q * a.pstride;
          const bool v = mv && p <= p_hi && q <= q_hi;  // windows that do not exist read zeros
          const int o = ((n * a.P + p) * a.Q + q) * C + ach * 8;
          rgd[i][2 * u + t] = buf_load16(dpr, v ? 2u * (unsigned)o : kOOB);
          rav[i][2 * u + t] = buf_load8(agr, v ? (unsigned)o : kOOB);
          me |= (unsigned)((r * a.PK + s) & 0xFF) << (8 * (2 * u + t));
        }
      rme[i] = me;
      ry[i] = buf_load16(yr, mv ? 2u * (unsigned)(m * C + ach * 8) : kOOB);
    }
    const int m = m0 + brow;
    const bool mv = m < mlim;
    const int n = mdiv(m, a.mag_hw), hw = m - n * HW;
    const int oh = mdiv(hw, a.mag_w), ow = hw - oh * a.W;
    const int ih0 = oh * a.stride - a.pad, iw0 = ow * a.stride - a.pad;
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int s = 2 * bc + p, ih = ih0 + j, iw = iw0 + s;
        const bool v = mv && j < a.R && s < a.S && (unsigned)ih < (unsigned)a.IH && (unsigned)iw < (unsigned)a.IW;
        rb[j][p] = buf_load8(xr, v ? 8u * (unsigned)((n * a.IH + ih) * a.IW + iw) : kOOB);
      }
  };
  // per-channel BN constants of this thread's channel group: re-read (L1 hits) per block instead of
  // pinning 40 VGPRs across the MFMAs
  int cbn = ach * 8;
  auto compute_store = [&](int buf) __attribute__((always_inline)) {
    if constexpr (!FUSED) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = arow + 32 * i;
        *reinterpret_cast<u32x4*>(sA + buf * BKM * C + row * C + (tr_swz(row, ach, 8) << 3)) = ry[i];
      }
    } else {
    asm volatile("" : "+v"(cbn));
    float s_[8], h_[8], k1[8], k2[8], k3[8];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const f32x4 v0 = *reinterpret_cast<const f32x4*>(a.sc + cbn + 4 * h);
      const f32x4 v1 = *reinterpret_cast<const f32x4*>(a.sh + cbn + 4 * h);
      const f32x4 v2 = *reinterpret_cast<const f32x4*>(a.coeff + cbn + 4 * h);
      const f32x4 v3 = *reinterpret_cast<const f32x4*>(a.coeff + C + cbn + 4 * h);
      const f32x4 v4 = *reinterpret_cast<const f32x4*>(a.coeff + 2 * C + cbn + 4 * h);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        s_[4 * h + j] = v0[j]; h_[4 * h + j] = v1[j]; k1[4 * h + j] = v2[j]; k2[4 * h + j] = v3[j];
        k3[4 * h + j] = v4[j];
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      float g[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int wdw = 0; wdw < 4; ++wdw) {
        float gv[8];
        unpack8(rgd[i][wdw], gv);
        const unsigned me = (rme[i] >> (8 * wdw)) & 0xFFu;
        const u32x2 av = rav[i][wdw];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const unsigned byte = ((j < 4 ? av.x : av.y) >> (8 * (j & 3))) & 0xFFu;
          g[j] += byte == me ? gv[j] : 0.f;
        }
      }
      float yv[8], o[8];
      unpack8(ry[i], yv);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float gm = (yv[j] * s_[j] + h_[j]) > 0.f ? g[j] : 0.f;
        o[j] = k1[j] * gm + k2[j] * yv[j] + k3[j];
      }
      const int row = arow + 32 * i;
      *reinterpret_cast<u32x4*>(sA + buf * BKM * C + row * C + (tr_swz(row, ach, 8) << 3)) = pack8(o);
    }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int cc = bc + 4 * j;
      *reinterpret_cast<u32x4*>(sB + buf * BKM * KT + brow * KT + (tr_swz(brow, cc, 32) << 3)) =
          u32x4{rb[j][0].x, rb[j][0].y, rb[j][1].x, rb[j][1].y};
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int g4 = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
  auto mma = [&](int buf) __attribute__((always_inline)) {
    const bf16* cA = sA + buf * BKM * C;
    const bf16* cB = sB + buf * BKM * KT;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int row = ks * 32 + 8 * g4 + q4, row2 = row + 4;
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int col = wm * 32 + i * 16 + 4 * p4;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (DBX_LDS s16x4*)(cA + row * C + (tr_swz(row, col >> 3, 8) << 3) + (col & 7)));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (DBX_LDS s16x4*)(cA + row2 * C + (tr_swz(row2, col >> 3, 8) << 3) + (col & 7)));
        af[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = wn * 128 + j * 16 + 4 * p4;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (DBX_LDS s16x4*)(cB + row * KT + (tr_swz(row, col >> 3, 32) << 3) + (col & 7)));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (DBX_LDS s16x4*)(cB + row2 * KT + (tr_swz(row2, col >> 3, 32) << 3) + (col & 7)));
        bfr[j] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };

  // branch-free pipeline: block kb+1's raw inputs load under block kb's MFMAs; past the last block
  // the loads read out of range and the staging fills the idle buffer (never read)
  load(0);
  compute_store(0);
  __syncthreads();
  for (int kb = 0; kb < nkb; ++kb) {
    load(kb + 1);
    mma(kb & 1);
    compute_store((kb + 1) & 1);
    __syncthreads();
  }
  // partial slab ws[split][c][kk] (kk = r*32 + s*4 + ci: the stem's 8 x 8 x 4 tap layout)
  float* out = a.ws + (size_t)split * C * KT;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = wm * 32 + i * 16 + g4 * 4 + r;
        out[(size_t)k * KT + wn * 128 + j * 16 + (lane & 15)] = acc[i][j][r];
      }
}

}  // namespace dbx

using namespace dbx;

// Returns the number of partial slabs written (= workgroups), or a negative error. fused = 0: the
// plain stem weight gradient of the stored gradient a.y (pool / BN fields unused).
extern "C" int dbx_stem_bwd(StemBwdArgs* args, long long ws_cap, int fused, hipStream_t st) {
  StemBwdArgs& a = *args;
  if (a.C != 64 || a.R > 8 || a.S > 8) return -40;
  if (fused && (a.PK + a.pstride - 1) / a.pstride > 2) return -41;  // <= 2 x 2 pooling windows per pixel
  if ((long long)a.N * a.H * a.W * a.C >= (1ll << 31) || 8ll * a.N * a.IH * a.IW >= (long long)kOOB) return -42;
  if (a.M <= 0) return -43;
  static const int cap = [] {
    int per_cu = 0, dev = 0, cus = 0;
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(&stem_bwd_kernel<true>),
                                                       256, 0);
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    return (per_cu > 0 && cus > 0) ? per_cu * cus : 256;
  }();
  const int nblk = (a.M + 63) / 64;
  int nsplit = nblk < cap ? nblk : cap;
  const int bps = (nblk + nsplit - 1) / nsplit;  // 64-pixel blocks per split
  a.m_per_split = bps * 64;
  nsplit = (nblk + bps - 1) / bps;
  a.nsplit = nsplit;
  if ((long long)(nsplit + (nsplit < 64 ? nsplit : 64)) * a.C * 256 > ws_cap) return -44;
  if (fused) hipLaunchKernelGGL(stem_bwd_kernel<true>, dim3(nsplit), dim3(256), 0, st, a);
  else hipLaunchKernelGGL(stem_bwd_kernel<false>, dim3(nsplit), dim3(256), 0, st, a);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? nsplit : -(int)e - 1000;
}
