// Eight-wave implicit-GEMM convolution for the compute-bound convs with plain operands (no BN
// prologue): forward (+ BN statistics epilogue) and stride-1 data gradients (+ the BN-backward
// epilogues) of the 3x3 convs at 28 / 14 / 7 and the 1x1 convs at 14 / 7, the ones the four-wave
// 128x128 kernel (conv_igemm_kernel.h) runs at 0.66-0.9 PF/s.
//
// Why a separate kernel (cdna_hip_programming.md §5, "the step-3 structure's ~900 TF ceiling"):
//   * a 256-row tile on 8 waves shares every staged weight (B) row across 256 output pixels and every
//     staged activation (A) row across BN = 128 / 256 channels: half the global->LDS bytes per FLOP of
//     the 128x128 tile, and for BN = 256 a 128x64 tile per wave (8 x 4 MFMA tiles, 0.375 ds_read_b128
//     per MFMA instead of 0.5);
//   * both operands move by LDS-DMA (buffer_load ... lds: no VGPR staging, no ds_write) through an
//     NBUF-slot ring: the DMA of K block kb + NBUF - 1 is in flight across the barrier of block kb
//     (counted vmcnt + raw s_barrier, never vmcnt(0) in the loop);
//   * inside a K block both k32 fragment sets are read before the first MFMA (24 / 16 ds_read_b128
//     in flight per wave), so the LDS latency hides under the other k-step's MFMAs and the second
//     wave of the SIMD;
//   * the MFMA bursts run at raised wave priority (s_setprio) so the sibling wave's LDS / DMA issue
//     interleaves with, instead of delaying, the matrix pipe.
// Tile geometry: 256 x BN x 64, 512 threads, one workgroup per CU (LDS: NBUF x (256 + BN) x 128 B),
// WM x WN = 2 x 4 (BN = 256) or 4 x 2 (BN = 128) waves. The epilogue is the shared igemm_epilogue
// (statistics on the matrix cores, BN-backward moments, residual-gradient accumulation).
#include "conv_igemm_kernel.h"

namespace dbx {

// BK: channels per ring stage -- 64 (NBUF 2 / 3), or 32 for the deep ring: with the 256 x 256 tile
// a 4-slot ring of 32-channel stages keeps three stages (3 x 1024 MFMA cycles per SIMD) in flight in
// the 128 KiB two 64-channel slots took (cdna_hip_programming.md §5, the 256^2 template's half-tile
// prefetch).
template <int BN, int MODE, bool STATS, bool ACCUM, int EPI, int NBUF, int BK = 64>
__global__ __launch_bounds__(512, 1) void fast_igemm_kernel(const IGemmArgs a) {
  constexpr int BM = 256, NT = 512, NW = 8;
  constexpr int WM = BN == 256 ? 2 : 4, WN = NW / WM;
  constexpr int TM = BM / (16 * WM), TN = BN / (16 * WN);
  constexpr int CPR = BK / 8;          // 16-B chunks per tile row
  constexpr int RPP = NT / CPR;        // tile rows per DMA pass (CPR lanes x 16 B per row)
  constexpr int A_CH = BM / RPP, B_CH = BN / RPP;
  static_assert(BK == 64 || BK == 32, "stage depth");
  constexpr int ND = A_CH + B_CH;      // DMA instructions per wave and K block
  constexpr int LDS_AB = NBUF * (BM + BN) * BK;
  constexpr int LDS_EP = BM * (BN + 8) + 2 * (3 * NW * BN);
  constexpr int LDS_MAIN = LDS_AB > LDS_EP ? LDS_AB : LDS_EP;
  static_assert(2 * LDS_MAIN <= 163840, "LDS");
  static_assert(MODE == FWD || MODE == DGRAD, "fast kernel: forward / data gradient");
  __shared__ __attribute__((aligned(16))) bf16 lds[LDS_MAIN];
  const bf16* sA = lds;                      // [NBUF][BM][BK]
  const bf16* sB = lds + NBUF * BM * BK;     // [NBUF][BN][BK]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wm = wid / WN, wn = wid % WN;
  const int ntn = a.OC / BN, ntm = (a.M + BM - 1) / BM, ntile = ntn * ntm;
  const int bid = xcd_remap(blockIdx.x, ntile);
  const int tm = bid / ntn, tn = bid - tm * ntn;
  const int m0 = tm * BM, n0 = tn * BN;

  // ---- A rows of this thread's DMA lanes: decompose the output pixel once -------------------
  const int ach = tid & (CPR - 1);
  const int lch = ach ^ fswz<BK>(tid / CPR);  // LDS position (row, ach) receives chunk lch (swizzle; RPP % 16 == 0)
  int ahb[A_CH], awb[A_CH];
  unsigned apix[A_CH];
#pragma unroll
  for (int i = 0; i < A_CH; ++i) {
    const int m = m0 + tid / CPR + RPP * i;
    const int ohw = a.OH * a.OW;
    int n = mdiv_or(m, a.mag_ohw, ohw);
    const int pq = m - n * ohw;
    const int oh = mdiv_or(pq, a.mag_ow, a.OW), ow = pq - oh * a.OW;
    if (m >= a.M) n = 0;
    if (MODE == DGRAD) { ahb[i] = oh + a.dh0; awb[i] = ow + a.dw0; }
    else { ahb[i] = oh * a.stride - a.pad; awb[i] = ow * a.stride - a.pad; }
    apix[i] = 2u * (unsigned)(((n * a.IH + ahb[i]) * a.IW + awb[i]) * a.IC + lch * 8);
    DBX_DCHECK(m >= a.M || (n >= 0 && n < a.N && oh >= 0 && oh < a.OH && ow >= 0 && ow < a.OW));
    if (m >= a.M) ahb[i] = -(1 << 28);
  }
  const int KTOT = a.R * a.S * a.IC;
  const int cpt = a.IC / BK;
  const int KB = a.nr * a.ns * cpt;
  const i32x4 xsrd = make_srd(a.x, 2ull * a.N * a.IH * a.IW * a.IC);
  const i32x4 wsrd = make_srd(a.w, 2ull * a.OC * KTOT);
  const unsigned lds0 = lds_addr(lds);
  // loader position (K block lk = (tap row ltr, tap column lts, channel block lcb)), advanced per issue
  int lk = 0, lcb = 0, lts = 0, ltr = 0;
  auto issue = [&](int slot) __attribute__((always_inline)) {
    const bool live = lk < KB;  // past the last block: out-of-range offsets (zeros into an idle slot)
    const int cb = lcb * BK;
    const int r = a.r0 + a.tstep * ltr, s = a.s0 + a.tstep * lts;
    const int dh = (MODE == DGRAD) ? -ltr : r, dw = (MODE == DGRAD) ? -lts : s;
    const unsigned toff = 2u * (unsigned)((dh * a.IW + dw) * a.IC + cb);
    const unsigned da = lds0 + 2u * (unsigned)(slot * BM * BK) + 1024u * (unsigned)wid;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const bool v = live && (unsigned)(ahb[i] + dh) < (unsigned)a.IH && (unsigned)(awb[i] + dw) < (unsigned)a.IW;
      lds_dma16(xsrd, v ? apix[i] + toff : kOOB, da + 1024u * (unsigned)(NW * i));
    }
    const int koff = (r * a.S + s) * a.IC + cb + lch * 8;
    const unsigned db = lds0 + 2u * (unsigned)(NBUF * BM * BK + slot * BN * BK) + 1024u * (unsigned)wid;
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int n = n0 + tid / CPR + RPP * i;
      lds_dma16(wsrd, live ? 2u * (unsigned)(n * KTOT + koff) : kOOB, db + 1024u * (unsigned)(NW * i));
    }
    ++lk;
    if (++lcb == cpt) { lcb = 0; if (++lts == a.ns) { lts = 0; ++ltr; } }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment reads of one stage from ring slot `slot`: both k32 steps of a 64-channel stage up front
  // (FS = 2), the one step of a 32-channel stage (FS = 1)
  constexpr int FS = BK / 32;
  bf16x8 fa[FS][TM], fb[FS][TN];
  auto read_frags = [&](int slot, int ks0, int nks) __attribute__((always_inline)) {
    const bf16* cA = sA + slot * BM * BK;
    const bf16* cB = sB + slot * BN * BK;
#pragma unroll
    for (int kq = 0; kq < nks; ++kq) {
      const int ks = (FS == 2) ? kq : 0;  // register set
      const int ch = (ks0 + kq) * 4 + (lane >> 4);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * (BN / WN) + j * 16 + (lane & 15);
        fb[ks][j] = *reinterpret_cast<const bf16x8*>(cB + row * BK + ((ch ^ fswz<BK>(row)) << 3));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * (BM / WM) + i * 16 + (lane & 15);
        fa[ks][i] = *reinterpret_cast<const bf16x8*>(cA + row * BK + ((ch ^ fswz<BK>(row)) << 3));
      }
    }
  };
  auto mma_step = [&](int kq) __attribute__((always_inline)) {
    const int ks = (FS == 2) ? kq : 0;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)  // C^T = W X^T: a lane's 4 accumulators = 4 channels of one pixel
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[ks][j], fa[ks][i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  // prologue: NBUF - 1 blocks in flight
#pragma unroll
  for (int sl = 0; sl < NBUF - 1; ++sl) issue(sl);
  int cur = 0;
  for (int kb = 0; kb < KB; ++kb) {
    dma_wait<(NBUF - 2) * ND>();  // this wave's part of block kb has landed (older than the newest NBUF-2)
    // every wave's part has landed, and every wave finished reading the slot the next issue refills
    // (its fragment reads completed: the MFMAs that consumed them were issued before this point)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    issue(cur == 0 ? NBUF - 1 : cur - 1);
    read_frags(cur, 0, FS);
#pragma unroll
    for (int kq = 0; kq < FS; ++kq) mma_step(kq);
    cur = cur + 1 == NBUF ? 0 : cur + 1;
  }
  dma_wait<0>();  // no DMA may still write the LDS the epilogue stages through
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
  igemm_epilogue<BM, BN, WM, WN, MODE, STATS, ACCUM, EPI>(a, acc, lds, m0, n0, tm, blockIdx.x);
}

}  // namespace dbx

using namespace dbx;

// 64-channel stages in a 2- (BN 256) / 3-slot (BN 128) ring. (Measured and removed in round 6: the deep
// ring of 32-channel stages (4 / 5 slots) and a ping-pong variant with staggered wave groups, neither
// faster in the step: profiles/r5_ring/, profiles/r4_s5/.)
template <int BN, int MODE, bool STATS, bool ACCUM, int EPI>
static int launch_fast(const IGemmArgs& a, hipStream_t st) {
  const int ntile = (a.OC / BN) * ((a.M + 255) / 256);
  hipLaunchKernelGGL((fast_igemm_kernel<BN, MODE, STATS, ACCUM, EPI, BN == 256 ? 2 : 3, 64>), dim3(ntile),
                     dim3(512), 0, st, a);
  return (int)hipGetLastError();
}

// bn: 128 | 256 (tile 256 x bn). FWD: stats only (no prologue / tail); DGRAD: no prologue / fold,
// any accumulate / epilogue (stride-1 geometry: one launch covers every output pixel).
extern "C" int dbx_conv_fast(int mode, int bn, const IGemmArgs* args, int stats, int accum, int epi, hipStream_t st) {
  const IGemmArgs& a = *args;
  if (a.IC % 64 != 0 || a.OC % bn != 0) return -60;
  if (a.in_scale || a.res) return -61;  // plain operands only
  if (mode == FWD) {
    if (accum || epi) return -62;
    if (bn == 256) return stats ? launch_fast<256, FWD, true, false, 0>(a, st) : launch_fast<256, FWD, false, false, 0>(a, st);
    if (bn == 128) return stats ? launch_fast<128, FWD, true, false, 0>(a, st) : launch_fast<128, FWD, false, false, 0>(a, st);
    return -63;
  }
  if (mode == DGRAD) {
    if (stats) return -62;
#define DBX_FAST_DG(BN_)                                                                       \
  if (epi == 0) return accum ? launch_fast<BN_, DGRAD, false, true, 0>(a, st)                  \
                             : launch_fast<BN_, DGRAD, false, false, 0>(a, st);               \
  if (epi == 1) return accum ? launch_fast<BN_, DGRAD, false, true, 1>(a, st)                  \
                             : launch_fast<BN_, DGRAD, false, false, 1>(a, st);
    if (bn == 256) {  // the MASK_Y epilogue next to 128 accumulators per lane spills (~95 VGPRs): 128-wide
      DBX_FAST_DG(256)
      return -66;
    }
    if (bn == 128) {
      DBX_FAST_DG(128)
      if (epi == 2) return accum ? launch_fast<128, DGRAD, false, true, 2>(a, st)
                                 : launch_fast<128, DGRAD, false, false, 2>(a, st);
    }
#undef DBX_FAST_DG
    return -63;
  }
  return -64;
}
