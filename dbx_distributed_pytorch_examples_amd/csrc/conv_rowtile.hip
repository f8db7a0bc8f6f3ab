// Row-tile kernel for the 1x1 stride-1 convs whose A operand carries a BN prologue and whose K is
// short next to N: the bottleneck's expanding conv3 forward (BN2-apply + ReLU prologue, BN3
// statistics epilogue, C -> 4C) and the folded conv1 data gradient (BN1-backward apply k1*g + k2*y +
// k3 while staging, residual-gradient accumulation + the block-input BN-backward epilogue, mid ->
// 4*mid). SURVEY.md §2.4 K2 / K4 / K6 / K7.
//
// In the implicit-GEMM kernel (conv_igemm_kernel.h) every N tile of an output row block re-reads the
// whole A row block (K channels of one or two tensors) and re-applies the prologue: at 14x14 / 7x7
// (N = 1024 / 2048 with K = 256 / 512) that is 4-8 L2 reads and transforms of every A element per
// output element written, and each tile pays the A-load latency before its short K loop (K / 64 = 1..8
// blocks). Here ONE workgroup owns a BM-row block for ALL N tiles:
//   1. A (BM x K) is loaded, transformed once (tail write-back: the applied operand once, not once
//      per N tile) and kept in LDS for the whole row block (K <= 256 at BM 128, <= 512 at BM 64);
//   2. the weights stream through a 3-slot LDS-DMA ring, one 64-channel block at a time in N-tile
//      order, two blocks ahead, so the next N tile's first blocks land during the current tile's
//      epilogue;
//   3. each N tile ends in the shared epilogue (igemm_epilogue: BN statistics on the matrix cores /
//      BN-backward moments, residual accumulate), staged in an LDS region of its own.
// Ring waits count only the DMA issued after the awaited block (dma_wait<ND>): epilogue stores
// younger than a prefetch make such a wait stricter, never weaker (vmcnt retires in order).
// 4 waves (2 x 2) of (BM/2) x (BN/2) output each; one workgroup per CU (LDS-bound); grid = row blocks.
#include "conv_igemm_kernel.h"

namespace dbx {

template <int BM, int BN, int KMAX, int MODE, bool TAIL, bool STATS, bool ACCUM, int EPI>
__global__ __launch_bounds__(256, 1) void rowtile_kernel(const IGemmArgs a) {
  constexpr int NT = 256, NW = 4, WM = 2, WN = 2, BK = 64, NBUF = 3;
  constexpr int TM = BM / (16 * WM), TN = BN / (16 * WN);
  constexpr int RPP = NT / 8;                  // rows per staging pass (8 lanes x 16 B per 64-ch row)
  constexpr int A_CH = BM / RPP, B_CH = BN / RPP;
  constexpr int ND = B_CH;                     // DMA instructions per wave and ring block
  constexpr int NPRO = TAIL ? 4 : 2;           // prologue affine arrays (scale, shift (, rs, rh))
  constexpr int LDS_A = KMAX * BM;             // resident transformed A: [K/64][BM][64]
  constexpr int LDS_B = NBUF * BN * BK;        // weight ring
  constexpr int LDS_E = BM * (BN + 8) + 2 * (3 * NW * BN);  // epilogue staging + reduction scratch
  constexpr int LDS_P = 2 * NPRO * KMAX;       // fp32 prologue coefficients (bf16 units)
  static_assert(2 * (LDS_A + LDS_B + LDS_E + LDS_P) <= 163840, "LDS");
  static_assert(MODE == FWD || TAIL, "the data-gradient row tile is the folded (BN-backward apply) one");
  __shared__ __attribute__((aligned(16))) bf16 lds[LDS_A + LDS_B + LDS_E + LDS_P];
  bf16* sA = lds;
  bf16* sB = lds + LDS_A;
  bf16* sE = sB + LDS_B;
  float* sPro = reinterpret_cast<float*>(sE + LDS_E);  // [NPRO][KMAX]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wm = wid / WN, wn = wid % WN;
  const int K = a.IC;                 // GEMM depth (1x1: the A tensor's channels), host-checked <= KMAX
  const int KB = K / BK;
  const int ntn = a.OC / BN;
  const int Q = ntn * KB;             // ring blocks of this row block (N-tile major)
  const int ntm = (a.M + BM - 1) / BM;
  const int tm = xcd_remap(blockIdx.x, ntm);
  const int m0 = tm * BM;

  // ---- prologue coefficients of all K channels --------------------------------------------
  for (int c = tid; c < K; c += NT) {
    sPro[c] = a.in_scale[c];
    sPro[KMAX + c] = a.in_shift[c];
    if constexpr (TAIL) {
      sPro[2 * KMAX + c] = a.res_scale ? a.res_scale[c] : 1.f;
      sPro[3 * KMAX + c] = a.res_shift ? a.res_shift[c] : 0.f;
    }
  }

  // ---- weight ring (block q = (N tile q / KB, K block q % KB)); past Q: out of range -> zeros ----
  const int ach = tid & 7;
  const int lch = ach ^ fswz<BK>(tid >> 3);  // source chunk of this lane's LDS position (RPP % 16 == 0)
  const i32x4 wsrd = make_srd(a.w, 2ull * a.OC * K);
  const unsigned lds0 = lds_addr(lds);
  auto issue = [&](int q, int slot) __attribute__((always_inline)) {
    const int nt = q / KB, kb = q - nt * KB;
    const bool live = q < Q;
    const unsigned dst = lds0 + 2u * (unsigned)(LDS_A + slot * BN * BK) + 1024u * (unsigned)wid;
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int n = nt * BN + (tid >> 3) + RPP * i;
      lds_dma16(wsrd, live ? 2u * (unsigned)(n * K + kb * BK + lch * 8) : kOOB, dst + 1024u * (unsigned)(NW * i));
    }
  };
  issue(0, 0);
  issue(1, 1);
  __syncthreads();  // sPro visible

  // ---- A: load, transform once, keep (2-deep register pipeline over the K blocks) -----------
  const rsrc_t xr = make_rsrc(a.x, 2ull * a.M * K);
  const rsrc_t rr_ = make_rsrc(a.res, TAIL ? 2ull * a.M * K : 0ull);
  const rsrc_t toutr = make_rsrc(a.tail_out, (TAIL && a.tail_out) ? 2ull * a.M * K : 0ull);
  const rsrc_t tbitr = make_rsrc(a.tail_bits, (TAIL && a.tail_bits) ? 1ull * a.M * K / 8 : 0ull);
  unsigned off[A_CH];
  bool rv[A_CH];
#pragma unroll
  for (int i = 0; i < A_CH; ++i) {
    const int m = m0 + (tid >> 3) + RPP * i;
    rv[i] = m < a.M;
    off[i] = 2u * (unsigned)(m * K + ach * 8);
  }
  u32x4 ra[2][A_CH], rr[2][TAIL ? A_CH : 1];
  auto load = [&](int kb, int S) __attribute__((always_inline)) {
    const bool live = kb < KB;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const unsigned o = (live && rv[i]) ? off[i] + 2u * (unsigned)(kb * BK) : kOOB;
      ra[S][i] = buf_load16(xr, o);
      if constexpr (TAIL) rr[S][i] = buf_load16(rr_, o);
    }
  };
  auto transform = [&](int kb, int S) __attribute__((always_inline)) {
    const int c0 = kb * BK + ach * 8;
    // one 4-channel half at a time (16 coefficient registers live, as the implicit-GEMM tail)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const f32x4 ps = *reinterpret_cast<const f32x4*>(sPro + c0 + 4 * h);
      const f32x4 ph = *reinterpret_cast<const f32x4*>(sPro + KMAX + c0 + 4 * h);
      f32x4 pr = {0.f, 0.f, 0.f, 0.f}, pq = {0.f, 0.f, 0.f, 0.f};
      if constexpr (TAIL) {
        pr = *reinterpret_cast<const f32x4*>(sPro + 2 * KMAX + c0 + 4 * h);
        pq = *reinterpret_cast<const f32x4*>(sPro + 3 * KMAX + c0 + 4 * h);
      }
#pragma unroll
      for (int i = 0; i < A_CH; ++i) {
        float f[4], g[4];
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          const unsigned xv = ra[S][i][2 * h + d];
          f[2 * d] = __uint_as_float(xv << 16); f[2 * d + 1] = __uint_as_float(xv & 0xFFFF0000u);
          if constexpr (TAIL) {
            const unsigned rvv = rr[S][i][2 * h + d];
            g[2 * d] = __uint_as_float(rvv << 16); g[2 * d + 1] = __uint_as_float(rvv & 0xFFFF0000u);
          }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          f[j] = f[j] * ps[j] + ph[j];
          if constexpr (TAIL) f[j] += g[j] * pr[j] + pq[j];  // as bn_apply / bn_bwd_apply compute it
        }
        ra[S][i][2 * h] = pack2(f[0], f[1]);
        ra[S][i][2 * h + 1] = pack2(f[2], f[3]);
      }
    }
    const u32x4 zero4 = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      u32x4 t = ra[S][i];
      if constexpr (MODE == FWD) t = relu_bf16x8(t);  // forward prologue: BN-apply + ReLU
      t = rv[i] ? t : zero4;                          // rows past M stay exactly zero
      const int row = (tid >> 3) + RPP * i;
      *reinterpret_cast<u32x4*>(sA + kb * BM * BK + row * BK + ((ach ^ fswz<BK>(row)) << 3)) = t;
      if constexpr (TAIL) {
        const unsigned o = rv[i] ? off[i] + 2u * (unsigned)(kb * BK) : kOOB;
        buf_store16(toutr, o, t);  // the applied operand (block output / BN-backward apply), once
        if constexpr (MODE == FWD) {
          unsigned bits = 0;
#pragma unroll
          for (int q = 0; q < 4; ++q)
            bits |= (((t[q] & 0xFFFFu) ? 1u : 0u) << (2 * q)) | (((t[q] >> 16) ? 1u : 0u) << (2 * q + 1));
          buf_store8(tbitr, o == kOOB ? kOOB : (o >> 4), (unsigned char)bits);
        }
      }
    }
  };
  load(0, 0);
  load(1, 1);
  for (int kb = 0; kb < KB; kb += 2) {
    transform(kb, 0);
    load(kb + 2, 0);
    if (kb + 1 < KB) {
      transform(kb + 1, 1);
      load(kb + 3, 1);
    }
  }
  dma_wait<0>();     // ring blocks 0, 1 (issued first) and everything the A phase issued
  __syncthreads();   // the resident A image and ring blocks 0 / 1 are visible to every wave

  // ---- N tiles: stream the weights, MFMA against the resident A, epilogue per tile ----------
  f32x4 acc[TM][TN];
  auto mma = [&](int kb, int slot) __attribute__((always_inline)) {
    const bf16* cA = sA + kb * BM * BK;
    const bf16* cB = sB + slot * BN * BK;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
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
        for (int j = 0; j < TN; ++j)  // C^T = W X^T: a lane's 4 accumulators are 4 channels of one pixel
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    }
  };
  int cur = 0;
  for (int q = 0; q < Q; ++q) {
    const int nt = q / KB, kb = q - nt * KB;
    if (kb == 0) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    if (q > 0) {
      dma_wait<ND>();   // this wave's part of block q landed (only block q+1's DMA may be younger... or
                        // stricter: epilogue stores younger than it retire too)
      __syncthreads();  // every wave's part; and slot (cur + 2) % 3 (block q - 1) is no longer read
    }
    issue(q + 2, cur == 0 ? 2 : cur - 1);
    mma(kb, cur);
    cur = cur == 2 ? 0 : cur + 1;
    if (kb == KB - 1)
      igemm_epilogue<BM, BN, WM, WN, MODE, STATS, ACCUM, EPI>(a, acc, sE, m0, nt * BN, tm, blockIdx.x);
  }
  dma_wait<0>();  // the past-the-end ring issues (zeros) have landed before the workgroup ends
}

}  // namespace dbx

using namespace dbx;

template <int BM, int BN, int KMAX, int MODE, bool TAIL, bool STATS, bool ACCUM, int EPI>
static int launch_rowtile(const IGemmArgs& a, hipStream_t st) {
  if (a.IC > KMAX || a.IC % 64 || a.OC % BN) return -71;
  const int ntm = (a.M + BM - 1) / BM;
  hipLaunchKernelGGL((rowtile_kernel<BM, BN, KMAX, MODE, TAIL, STATS, ACCUM, EPI>), dim3(ntm), dim3(256), 0, st, a);
  return (int)hipGetLastError();
}

// The row-tile kernel (tune-table tile code 7): 1x1 stride-1 convs only. FWD: BN prologue (+ tail),
// statistics epilogue; DGRAD: the folded BN-backward apply (a.res set), accumulate / EPI 0-2. BM 128
// for K <= 256, BM 64 for K <= 512 (the resident A image).
#define DBX_RT(BM_, KM_)                                                                                   \
  if (mode == FWD) {                                                                                       \
    if (!stats) return -72;                                                                                \
    return a.res ? launch_rowtile<BM_, 128, KM_, FWD, true, true, false, 0>(a, st)                         \
                 : launch_rowtile<BM_, 128, KM_, FWD, false, true, false, 0>(a, st);                       \
  }                                                                                                        \
  if (accum) {                                                                                             \
    if (epi == 1) return launch_rowtile<BM_, 128, KM_, DGRAD, true, false, true, 1>(a, st);                \
    if (epi == 0) return launch_rowtile<BM_, 128, KM_, DGRAD, true, false, true, 0>(a, st);                \
    return -73;                                                                                            \
  }                                                                                                        \
  if (epi == 2) return launch_rowtile<BM_, 128, KM_, DGRAD, true, false, false, 2>(a, st);                 \
  if (epi == 0) return launch_rowtile<BM_, 128, KM_, DGRAD, true, false, false, 0>(a, st);                 \
  return -73;

extern "C" int dbx_conv_rowtile(int mode, const IGemmArgs* args, int stats, int accum, int epi, hipStream_t st) {
  const IGemmArgs& a = *args;
  if (a.R != 1 || a.S != 1 || a.stride != 1 || a.pad != 0 || !a.in_scale) return -70;
  if (mode == DGRAD && (!a.res || a.osub != 1 || a.add_sub > 1)) return -70;
  if (mode == FWD && !a.relu_in) return -70;
  if (a.IC <= 256) { DBX_RT(128, 256) }
  if (a.IC <= 512) { DBX_RT(64, 512) }
  return -71;
}
#undef DBX_RT
