// Implicit-GEMM conv entry points: forward / stem dispatch, weight gradients, split-K reduction.
// The igemm_kernel template lives in conv_igemm_kernel.h; the dgrad instantiations are compiled
// in conv_dgrad.hip (a separate translation unit, so the two compile in parallel).
#include "conv_igemm_kernel.h"

namespace dbx {

// ======================================================================================
// Weight gradient: dW[k][kk] = sum_m dY[m][k] * Xcol[m][kk]   (kk = (r, s, c), KRSC order)
// Both operands arrive pixel-major (reduction dim outermost), so tiles are staged as
// [64 pixels][128 cols] row-major (16B/lane copies) and the MFMA fragments are read
// column-wise with ds_read_b64_tr_b16 (gfx950 hardware-transposed LDS read). The reduction over
// M = N*OH*OW (up to 3.2M pixels) is split over blocks; each block writes an fp32 partial slab
// and wgrad_reduce sums the slabs in a fixed order (deterministic).
// ======================================================================================

// End of a weight-gradient tile: the fp32 partial slab ws[split][k][kk], or (a.dw set) the finished
// gradient. With one split the tile is written to dw straight from the accumulators. Otherwise the
// in-launch split-K reduction (cdna_hip_programming.md §5, "Projection GEMM at M = 256" item 2, in
// its write-through form): every block stores its partial tile with 16-B sc1 (write-through) buffer
// stores in the accumulators' own lane order -- tile region ((split * ntile + tile) * BM * BN) -- so
// no release fence (a buffer_wbl2 per block) is needed; each wave drains its stores, then one lane
// takes a relaxed agent-scope ticket from cnt[tile]; the block drawing nsplit-1 loads the nsplit
// partials of the tile with sc1 loads at the same lane positions (/opt/skills/guides/MI355X_MICROARCH.md, the image's CDNA4 guide, "Valid forms",
// row 1) and sums them in split order -- the same fp32 order per element as wgrad_reduce_kernel, so
// the result is bit-identical to the two-kernel path when that sums in one level -- and writes dw;
// then resets the counter. The host enables it only when a tile's partials are small (the reducer
// reads nsplit x BM x BN x 4 bytes alone).
template <int BM, int BN, int WM, int WN, int TM, int TN>
__device__ __forceinline__ void wgrad_store(const WgradArgs& a, f32x4 (&acc)[TM][TN], const int split,
                                            const int tile, const int k0, const int kk0, bf16* lds) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wm = wid / WN, wn = wid % WN;
  if (a.dw != nullptr && a.nsplit == 1) {  // uniform: the finished gradient straight from the tile
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      // one accumulator row at a time: without the fence the compiler hoists every dw load of the
      // accumulate path ahead of the stores (TM x TN x 4 more live registers: spills at 256 x 256)
      asm volatile("" ::: "memory");
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int k = k0 + wm * (BM / WM) + i * 16 + (lane >> 4) * 4 + r;
          const int kk = kk0 + wn * (BN / WN) + j * 16 + (lane & 15);
          const size_t e = (size_t)k * a.KTOT + kk;
          float v = acc[i][j][r] * a.scale;
          if (a.accumulate) v += a.dw[e];
          a.dw[e] = v;
        }
    }
    return;
  }
  if (a.dw == nullptr) {  // slab for the separate reduce kernel: ws[split][k][kk]
    float* out = a.ws + (size_t)split * a.OC * a.KTOT;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int k = k0 + wm * (BM / WM) + i * 16 + (lane >> 4) * 4 + r;
          const int kk = kk0 + wn * (BN / WN) + j * 16 + (lane & 15);
          out[(size_t)k * a.KTOT + kk] = acc[i][j][r];
        }
    return;
  }
  const int ntile = (a.OC / BM) * (a.KTOT / BN);
  const rsrc_t ws = make_rsrc(a.ws, (unsigned long long)a.nsplit * ntile * BM * BN * 4);
  // this thread's 16-B slot of accumulator (i, j) inside a tile region
  auto slot = [&](int s, int i, int j) __attribute__((always_inline)) {
    return (unsigned)((((size_t)s * ntile + tile) * BM * BN + ((size_t)(wid * TM + i) * TN + j) * 256 + lane * 4) * 4);
  };
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned,
                                                                acc[i][j]),
                                             ws, slot(split, i, j), 0, 16);  // aux 16: sc1 (write-through)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's partial has reached memory
  __syncthreads();                                   // ... every wave's; LDS no longer read
  int* flag = reinterpret_cast<int*>(lds);
  if (tid == 0) {
    const unsigned t = __hip_atomic_fetch_add((gu32*)(a.cnt + tile), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    flag[0] = t == (unsigned)(a.nsplit - 1);
  }
  __syncthreads();
  if (!flag[0]) return;  // block-uniform
  f32x4 (&s)[TM][TN] = acc;  // the partials are stored: reuse the accumulator registers for the sum
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
      s[i][j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(ws, slot(0, i, j), 0, 16));
  for (int k = 1; k < a.nsplit; ++k) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        s[i][j] += __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(ws, slot(k, i, j), 0, 16));
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = k0 + wm * (BM / WM) + i * 16 + (lane >> 4) * 4 + r;
        const int kk = kk0 + wn * (BN / WN) + j * 16 + (lane & 15);
        const size_t e = (size_t)k * a.KTOT + kk;
        float v = s[i][j][r] * a.scale;
        if (a.accumulate) v += a.dw[e];
        a.dw[e] = v;
        asm volatile("" ::: "memory");
      }
  if (tid == 0) __hip_atomic_store((gu32*)(a.cnt + tile), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// WM x WN waves (64*WM*WN threads), each owning a (BM/WM) x (BN/WN) block of dW.
template <int BM, int BN, int WM, int WN, int MODE, bool PRO, int DEPTH = 2>
__global__ __launch_bounds__(64 * WM * WN, 2) void wgrad_kernel(const WgradArgs a) {
  constexpr int NT = 64 * WM * WN;
  constexpr int BKM = 64;                    // pixels per K block
  constexpr int NCA = BM / 8, NCB = BN / 8;  // 16B chunks per tile row
  constexpr int A_CH = BKM * NCA / NT, B_CH = BKM * NCB / NT;
  constexpr int TM = BM / (16 * WM), TN = BN / (16 * WN);
  __shared__ __attribute__((aligned(16))) bf16 lds[2 * BKM * (BM + BN) + (PRO ? 4 * BN : 0)];
  bf16* sA = lds;                   // [2][BKM][BM]
  bf16* sB = lds + 2 * BKM * BM;    // [2][BKM][BN]
  float* sPro = reinterpret_cast<float*>(lds + 2 * BKM * (BM + BN));  // [2][BN] prologue scale, shift

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wm = wid / WN, wn = wid % WN;
  const int ntm = a.OC / BM, ntn = a.KTOT / BN;
  const int ntile = ntm * ntn;
  // logical id = split * ntile + tile: consecutive ids share a split's dY / X rows, and the XCD
  // remap keeps consecutive ids on one XCD so those rows are fetched into ONE L2, not eight
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = bid / ntile;
  const int tile = bid - split * ntile;
  const int tm = tile / ntn, tn = tile - (tile / ntn) * ntn;
  const int k0 = tm * BM, kk0 = tn * BN;
  const int mbeg = split * a.m_per_split;
  const int mend = min(a.M, mbeg + a.m_per_split);
  const int nkb = (mend - mbeg + BKM - 1) / BKM;

  // A (dY) loader: thread -> (pixel row a_row, chunk column a_c)
  // each thread owns one pixel row and A_CH chunks of it (chunk = c0 + j*stride)
  constexpr int ATPR = NCA / A_CH;   // threads per pixel row for A
  constexpr int BTPR = NCB / B_CH;   // threads per pixel row for B
  const int a_row = tid / ATPR, a_c = tid % ATPR;
  const int b_row = tid / BTPR, b_c = tid % BTPR;

  // B column chunks: tap and channel per chunk (fixed over the K loop), and the chunk's element
  // offset relative to the receptive field's top-left pixel (32-bit)
  int b_tap_h[B_CH], b_tap_w[B_CH], b_ch[B_CH], b_off[B_CH];
#pragma unroll
  for (int j = 0; j < B_CH; ++j) {
    const int cc = b_c + j * BTPR;
    const int kk = kk0 + cc * 8;
    if constexpr (MODE == STEM) {  // kk = r*32 + s*4 + c  (8 pixels x 4 ch per filter row)
      b_tap_h[j] = kk >> 5; b_tap_w[j] = (kk >> 2) & 7; b_ch[j] = 0;
    } else {
      const int tap = kk / a.IC;
      b_ch[j] = kk - tap * a.IC;
      b_tap_h[j] = tap / a.S; b_tap_w[j] = tap - (tap / a.S) * a.S;
    }
    b_off[j] = (b_tap_h[j] * a.IW + b_tap_w[j]) * a.IC + b_ch[j];
  }
  // Two register staging sets (the K loop is unrolled by two so S is a constant): block kb+2 is
  // loaded while block kb+1's set is still landing, so each load has two blocks of MFMA work to
  // hide behind. The prologue affine of the tile's BN columns lives in LDS, not in registers.
  u32x4 ra[2][A_CH], rb[2][B_CH];
  const u32x4 zero4 = {0u, 0u, 0u, 0u};
  unsigned bvalid[2] = {0u, 0u};  // bit j: B chunk j is a real (non-padding) tap (PRO only)
  if constexpr (PRO) {
    for (int c = tid; c < BN; c += NT) {
      const int kk = kk0 + c;
      const int ch = kk - (kk / a.IC) * a.IC;
      sPro[c] = a.in_scale[ch];
      sPro[BN + c] = a.in_shift[ch];
    }
  }

  const rsrc_t dyr = make_rsrc(a.dy, 2ull * a.M * a.OC);
  const rsrc_t xr = make_rsrc(a.x, 2ull * a.N * a.IH * a.IW * a.IC);
  auto load = [&](int kb, int S) __attribute__((always_inline)) {
    // dY rows past the split read out of range (zeros): they add nothing to the reduction
    const int ma = mbeg + kb * BKM + a_row;
    const bool av = ma < mend;
#pragma unroll
    for (int j = 0; j < A_CH; ++j) {
      const int cc = a_c + j * ATPR;
      ra[S][j] = buf_load16(dyr, av ? 2u * (unsigned)(ma * a.OC + k0 + cc * 8) : kOOB);
    }
    const int mb = mbeg + kb * BKM + b_row;
    const bool mv = mb < mend;
    const int ohw = a.OH * a.OW;
    const int n = mv ? mdiv(mb, a.mag_ohw) : 0;
    const int pq = mb - n * ohw;
    const int oh = mdiv(pq, a.mag_ow), ow = pq - oh * a.OW;
    const bf16* base = a.x + (size_t)n * a.IH * a.IW * a.IC;
    const int ih0 = oh * a.stride - a.pad, iw0 = ow * a.stride - a.pad;
    const unsigned pix = 2u * (unsigned)(((n * a.IH + ih0) * a.IW + iw0) * a.IC);
    bvalid[S] = 0;
#pragma unroll
    for (int j = 0; j < B_CH; ++j) {
      const int ih = ih0 + b_tap_h[j];
      if constexpr (MODE == STEM) {
        // 16B chunk = 2 pixels (s, s+1) x 4 channels
        unsigned int w4[4];
        const bool rv = mv && b_tap_h[j] < a.R && ih >= 0 && ih < a.IH;
#pragma unroll
        for (int p = 0; p < 2; ++p) {  // branch-free (see the stem A loader in igemm_kernel)
          const int s = b_tap_w[j] + p, iw = ow * a.stride - a.pad + s;
          const bool v = rv && s < a.S && (unsigned)iw < (unsigned)a.IW;
          const uint2 t = *reinterpret_cast<const uint2*>(base + (v ? (ih * a.IW + iw) * 4 : 0));
          w4[2 * p] = v ? t.x : 0u; w4[2 * p + 1] = v ? t.y : 0u;
        }
        rb[S][j] = u32x4{w4[0], w4[1], w4[2], w4[3]};
      } else {
        const int iw = iw0 + b_tap_w[j];
        const bool v = mv && (unsigned)ih < (unsigned)a.IH && (unsigned)iw < (unsigned)a.IW;
        // padding taps / pixels past the split read out of range: zeros from the hardware
        rb[S][j] = buf_load16(xr, v ? pix + 2u * (unsigned)b_off[j] : kOOB);
        if constexpr (PRO) bvalid[S] |= (v ? 1u : 0u) << j;
      }
    }
  };
  // BN-apply (+ReLU) on the staged x chunks, after the MFMAs of the current block so the next
  // blocks' loads stay in flight meanwhile; padding taps stay exactly zero.
  auto pro_b = [&](int S) __attribute__((always_inline)) {
    if constexpr (PRO && MODE != STEM) {
#pragma unroll
      for (int j = 0; j < B_CH; ++j) {
        const int c = (b_c + j * BTPR) * 8;
        const f32x4 s0 = *reinterpret_cast<const f32x4*>(sPro + c);
        const f32x4 s1 = *reinterpret_cast<const f32x4*>(sPro + c + 4);
        const f32x4 h0 = *reinterpret_cast<const f32x4*>(sPro + BN + c);
        const f32x4 h1 = *reinterpret_cast<const f32x4*>(sPro + BN + c + 4);
        float f[8];
        unpack8(rb[S][j], f);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          f[e] = f[e] * s0[e] + h0[e];
          f[e + 4] = f[e + 4] * s1[e] + h1[e];
        }
        u32x4 t = pack8(f);
        t = relu_bf16x8(t);  // PRO implies ReLU (host-checked)
        rb[S][j] = ((bvalid[S] >> j) & 1u) ? t : zero4;
      }
    }
  };
  auto store = [&](int buf, int S) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < A_CH; ++j) {
      const int cc = a_c + j * ATPR;
      *reinterpret_cast<u32x4*>(sA + buf * BKM * BM + a_row * BM + (tr_swz(a_row, cc, NCA) << 3)) = ra[S][j];
    }
#pragma unroll
    for (int j = 0; j < B_CH; ++j) {
      const int cc = b_c + j * BTPR;
      *reinterpret_cast<u32x4*>(sB + buf * BKM * BN + b_row * BN + (tr_swz(b_row, cc, NCB) << 3)) = rb[S][j];
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  auto mma = [&](int buf) __attribute__((always_inline)) {
    const bf16* cA = sA + buf * BKM * BM;
    const bf16* cB = sB + buf * BKM * BN;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int col = wm * (BM / WM) + i * 16 + 4 * p;
        s16x4 lo, hi;
        {
          const int row = ks * 32 + 8 * g + q;
          lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (DBX_LDS s16x4*)(cA + row * BM + (tr_swz(row, col >> 3, NCA) << 3) + (col & 7)));
          const int row2 = row + 4;
          hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (DBX_LDS s16x4*)(cA + row2 * BM + (tr_swz(row2, col >> 3, NCA) << 3) + (col & 7)));
        }
        af[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = wn * (BN / WN) + j * 16 + 4 * p;
        s16x4 lo, hi;
        {
          const int row = ks * 32 + 8 * g + q;
          lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (DBX_LDS s16x4*)(cB + row * BN + (tr_swz(row, col >> 3, NCB) << 3) + (col & 7)));
          const int row2 = row + 4;
          hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (DBX_LDS s16x4*)(cB + row2 * BN + (tr_swz(row2, col >> 3, NCB) << 3) + (col & 7)));
        }
        bfr[j] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };
  // branch-free pipeline (see igemm_kernel): unconditional clamped prefetch, peeled odd tail
  auto step = [&](int kb, int S) __attribute__((always_inline)) {
    if constexpr (DEPTH == 2) {
      load(kb + 2 < nkb ? kb + 2 : nkb - 1, S ^ 1);
      mma(kb & 1);
      pro_b(S);
      store((kb + 1) & 1, S);
    } else {
      load(kb + 1 < nkb ? kb + 1 : nkb - 1, 0);
      mma(kb & 1);
      pro_b(0);
      store((kb + 1) & 1, 0);
    }
    __syncthreads();
  };
  __syncthreads();  // sPro visible
  if (nkb > 0) {
    load(0, 0);
    if (DEPTH == 2) load(nkb > 1 ? 1 : 0, 1);
    pro_b(0);
    store(0, 0);
    __syncthreads();
    int kb = 0;
    for (; kb + 1 < nkb; kb += 2) {
      step(kb, 1);
      step(kb + 1, DEPTH == 2 ? 0 : 1);
    }
    if (kb < nkb) mma(kb & 1);
  }
  wgrad_store<BM, BN, WM, WN, TM, TN>(a, acc, split, tile, k0, kk0, lds);
}

// Weight gradient without a BN prologue, operands moved by LDS-DMA (common.h lds_dma16): each
// wave-instruction fills 1 KiB of a tile image straight from memory, so the K loop has no
// register staging and no ds_write -- only the transposed fragment reads and the MFMAs touch
// the LDS port. The swizzle moves to the source side: LDS position p of a tile image (row =
// pixel p / NC, position p % NC) receives chunk tr_swz(row, p % NC) of that pixel (tr_swz is an
// XOR, its own inverse), so the fragment reads are those of wgrad_kernel unchanged.
// NBUF-deep ring: block kb+NBUF-1 is issued while block kb is computed; at the top of each step
// the wave waits until only the younger blocks' DMAs are in flight, then one barrier publishes
// every wave's part of block kb and retires the buffer the next issue overwrites.
// BKM: pixels per ring slot (64, or 32 for the 256 x 256 tile: its 4-slot ring keeps three 32-pixel
// stages in flight in 128 KiB, one barrier per stage). The 256 x 256 tile runs 2 x 4 waves of 128 x 64
// (8 x 4 MFMA tiles: 0.375 fragment reads per MFMA instead of 0.5, half the staged bytes per FLOP of
// 256 x 128) at one workgroup per CU with the whole register file.
template <int BM, int BN, int WM, int WN, int NBUF, int BKM = 64>
__global__ __launch_bounds__(64 * WM * WN, (BM * BN >= 256 * 256) ? 1 : 2) void wgrad_dma_kernel(const WgradArgs a) {
  constexpr int NT = 64 * WM * WN, NW = WM * WN;
  static_assert(BKM == 32 || BKM == 64, "pixels per stage");
  constexpr int NCA = BM / 8, NCB = BN / 8;
  constexpr int DA = BKM * NCA / NT, DB = BKM * NCB / NT;  // DMA instructions per wave and block
  constexpr int ND = DA + DB;
  constexpr int TM = BM / (16 * WM), TN = BN / (16 * WN);
  constexpr int IMG = BKM * (BM + BN);  // bf16 elements per ring slot
  static_assert(DA >= 1 && DB >= 1 && (NBUF - 1) * ND < 64, "tile / ring shape");
  __shared__ __attribute__((aligned(1024))) bf16 lds[NBUF * IMG];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wm = wid / WN, wn = wid % WN;
  const int ntn = a.KTOT / BN;
  const int ntile = (a.OC / BM) * ntn;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = bid / ntile;
  const int tile = bid - split * ntile;
  const int tm = tile / ntn, tn = tile - tm * ntn;
  const int k0 = tm * BM, kk0 = tn * BN;
  const int mbeg = split * a.m_per_split;
  const int mend = min(a.M, mbeg + a.m_per_split);
  const int nkb = (mend - mbeg + BKM - 1) / BKM;

  // per DMA instruction j: the pixel row inside the block and the source chunk (swizzle inverse).
  // A (dy rows): a_base[j] = the row's element offset relative to the block's first pixel.
  // B (im2col of x): the source position is carried from block to block instead of re-derived --
  // packed (oh << 16 | ow) of the row's pixel and the element offset of its tap, advanced by the
  // block's BKM pixels as a mixed-radix add (carries ow -> oh -> n), so the issue path has no
  // pixel -> (n, oh, ow) divisions (40+ quarter-rate multiplies per block and wave before).
  int a_row[DA], a_base[DA], b_row[DB], b_off[DB];
  unsigned b_pos[DB], b_tap[DB];  // (oh << 16) | ow ; (th << 16) | tw
#pragma unroll
  for (int j = 0; j < DA; ++j) {
    const int p = (j * NW + wid) * 64 + lane;
    a_row[j] = p / NCA;
    a_base[j] = a_row[j] * a.OC + k0 + tr_swz(a_row[j], p % NCA, NCA) * 8;
  }
  const int ohw = a.OH * a.OW;
#pragma unroll
  for (int j = 0; j < DB; ++j) {
    const int p = (j * NW + wid) * 64 + lane;
    b_row[j] = p / NCB;
    const int kk = kk0 + tr_swz(b_row[j], p % NCB, NCB) * 8;
    const int tap = kk / a.IC, ch = kk - (kk / a.IC) * a.IC;
    const int th = tap / a.S, tw = tap - (tap / a.S) * a.S;
    b_tap[j] = ((unsigned)th << 16) | (unsigned)tw;
    const int mb = mbeg + b_row[j];  // the row's pixel in block 0 (mb < 2^31: any value decomposes)
    const int n = mdiv(mb, a.mag_ohw);
    const int pq = mb - n * ohw;
    const int oh = mdiv(pq, a.mag_ow), ow = pq - oh * a.OW;
    b_pos[j] = ((unsigned)oh << 16) | (unsigned)ow;
    b_off[j] = ((n * a.IH + oh * a.stride - a.pad + th) * a.IW + ow * a.stride - a.pad + tw) * a.IC + ch;
  }
  // one block = BKM pixels = s_n images + s_oh rows + s_ow columns (s_oh < OH, s_ow < OW)
  const int s_ow = BKM % a.OW, s_oh = (BKM / a.OW) % a.OH, s_n = BKM / ohw;
  const unsigned pinc = ((unsigned)s_oh << 16) | (unsigned)s_ow;
  const int d0 = (s_n * a.IH * a.IW + (s_oh * a.IW + s_ow) * a.stride) * a.IC;  // no carry
  const int d1 = (a.IW - a.OW) * a.stride * a.IC;                               // ow wrapped: next row
  const int d2 = (a.IH - a.OH * a.stride) * a.IW * a.IC;                        // oh wrapped: next image
  const i32x4 dyr = make_srd(a.dy, 2ull * a.M * a.OC);
  const i32x4 xr = make_srd(a.x, 2ull * a.N * a.IH * a.IW * a.IC);
  const unsigned lbase = lds_addr(lds);

  // issue block kb (the next block in order: every call advances the B positions by one block) into
  // ring slot s; rows past the split / blocks past the end read out of range: zeros, no traffic.
  // Branch-free: every address is computed, the validity only selects kOOB.
  auto issue = [&](int kb, int s) __attribute__((always_inline)) {
    const unsigned sa = lbase + 2u * (unsigned)(s * IMG);
    const unsigned sb = sa + 2u * (unsigned)(BKM * BM);
    const int m0 = mbeg + kb * BKM;
    const int rows = (kb < nkb ? mend : 0) - m0;  // wave-uniform: rows of this block inside the split
#pragma unroll
    for (int j = 0; j < DA; ++j) {
      const unsigned off = a_row[j] < rows ? 2u * (unsigned)(m0 * a.OC + a_base[j]) : kOOB;
      lds_dma16(dyr, off, sa + 1024u * (unsigned)(j * NW + wid));
    }
#pragma unroll
    for (int j = 0; j < DB; ++j) {
      const int ih = __mul24((int)(b_pos[j] >> 16), a.stride) - a.pad + (int)(b_tap[j] >> 16);
      const int iw = __mul24((int)(b_pos[j] & 0xFFFFu), a.stride) - a.pad + (int)(b_tap[j] & 0xFFFFu);
      const bool v = b_row[j] < rows && (unsigned)ih < (unsigned)a.IH && (unsigned)iw < (unsigned)a.IW;
      lds_dma16(xr, v ? 2u * (unsigned)b_off[j] : kOOB, sb + 1024u * (unsigned)(j * NW + wid));
      // advance to the same row of the next block
      unsigned pos = b_pos[j] + pinc;
      const bool c1 = (int)(pos & 0xFFFFu) >= a.OW;
      pos += c1 ? 0x10000u - (unsigned)a.OW : 0u;
      const bool c2 = (int)(pos >> 16) >= a.OH;
      pos -= c2 ? (unsigned)a.OH << 16 : 0u;
      b_pos[j] = pos;
      b_off[j] += d0 + (c1 ? d1 : 0) + (c2 ? d2 : 0);
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  auto mma = [&](int s) __attribute__((always_inline)) {
    const bf16* cA = lds + s * IMG;
    const bf16* cB = cA + BKM * BM;
#pragma unroll
    for (int ks = 0; ks < BKM / 32; ++ks) {
      const int row = ks * 32 + 8 * g + q, row2 = row + 4;
      auto frag_a = [&](int i) __attribute__((always_inline)) {
        const int col = wm * (BM / WM) + i * 16 + 4 * p;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (DBX_LDS s16x4*)(cA + row * BM + (tr_swz(row, col >> 3, NCA) << 3) + (col & 7)));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (DBX_LDS s16x4*)(cA + row2 * BM + (tr_swz(row2, col >> 3, NCA) << 3) + (col & 7)));
        return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      };
      bf16x8 bfr[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = wn * (BN / WN) + j * 16 + 4 * p;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (DBX_LDS s16x4*)(cB + row * BN + (tr_swz(row, col >> 3, NCB) << 3) + (col & 7)));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (DBX_LDS s16x4*)(cB + row2 * BN + (tr_swz(row2, col >> 3, NCB) << 3) + (col & 7)));
        bfr[j] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
      if constexpr (BM * BN >= 256 * 256) {
        // 128 accumulators per lane: A fragments two at a time (register budget), the MFMA bursts at
        // raised priority ahead of the sibling wave's fragment reads and DMA issue
        bf16x8 a0 = frag_a(0), a1 = frag_a(1);
#pragma unroll
        for (int i = 0; i < TM; i += 2) {
          const bf16x8 c0 = a0, c1 = a1;
          if (i + 2 < TM) { a0 = frag_a(i + 2); a1 = frag_a(i + 3); }
          __builtin_amdgcn_s_setprio(1);
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(c0, bfr[j], acc[i][j], 0, 0, 0);
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i + 1][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(c1, bfr[j], acc[i + 1][j], 0, 0, 0);
          __builtin_amdgcn_s_setprio(0);
        }
      } else {
        bf16x8 af[TM];
#pragma unroll
        for (int i = 0; i < TM; ++i) af[i] = frag_a(i);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    }
  };

  // prologue: blocks 0 .. NBUF-2 in flight
#pragma unroll
  for (int s = 0; s < NBUF - 1; ++s) issue(s, s);
  int cur = 0;  // ring slot of block kb; block kb + NBUF - 1 goes to slot (cur + NBUF - 1) % NBUF
  for (int kb = 0; kb < nkb; ++kb) {
    dma_wait<(NBUF - 2) * ND>();  // this wave's part of block kb has landed
    __syncthreads();              // ... every wave's; and slot cur-1 is no longer read
    const int nxt = cur == 0 ? NBUF - 1 : cur - 1;
    issue(kb + NBUF - 1, nxt);
    mma(cur);
    cur = cur + 1 == NBUF ? 0 : cur + 1;
  }
  dma_wait<0>();  // no DMA may still be writing LDS when the wave ends
  wgrad_store<BM, BN, WM, WN, TM, TN>(a, acc, split, tile, k0, kk0, lds);
}

// Deterministic 2-level split-K reduction. Level 1 (G > 1): thread (i, g) sums the fixed split
// range of group g into ws2[g][i]; level 2 sums the G group partials in order, scales, and writes
// (or accumulates into) the fp32 gradient. Both levels are wide (n4 x G threads), so a 1024-split
// reduction of a tiny 64x64 weight no longer serialises 1024 dependent loads in one thread.
// s + slab(k0) + slab(k0 + 1) + ... + slab(k1 - 1), added strictly in that order (the fixed-order,
// deterministic split-K sum) with the loads issued eight at a time ahead of their adds: the reduces
// are latency-bound chains of dependent slab loads on the small (launch-bound) steps.
template <class T, class F>
__device__ __forceinline__ T sum_slabs_in_order(T s, int k0, int k1, F load) {
  int k = k0;
  for (; k + 8 <= k1; k += 8) {
    T v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = load(k + j);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += v[j];
  }
  for (; k < k1; ++k) s += load(k);
  return s;
}

__global__ void wgrad_reduce_l1_kernel(const float* __restrict__ ws, float* __restrict__ ws2, int n4, int nsplit,
                                       int spg) {
  const f32x4* w4 = reinterpret_cast<const f32x4*>(ws);
  f32x4* o4 = reinterpret_cast<f32x4*>(ws2);
  const int g = blockIdx.y;
  const int s0 = g * spg, s1 = min(nsplit, s0 + spg);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += gridDim.x * blockDim.x) {
    const f32x4 s = sum_slabs_in_order(f32x4{0.f, 0.f, 0.f, 0.f}, s0, s1,
                                       [&](int k) { return w4[(size_t)k * n4 + i]; });
    o4[(size_t)g * n4 + i] = s;
  }
}
__global__ void wgrad_reduce_kernel(const float* __restrict__ ws, float* __restrict__ dw,
                                    int n4, int nsplit, float scale, int accumulate) {
  const f32x4* w4 = reinterpret_cast<const f32x4*>(ws);
  f32x4* o4 = reinterpret_cast<f32x4*>(dw);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += gridDim.x * blockDim.x) {
    f32x4 s = sum_slabs_in_order(w4[i], 1, nsplit, [&](int k) { return w4[(size_t)k * n4 + i]; });
    s *= scale;
    if (accumulate) s += o4[i];
    o4[i] = s;
  }
}

// Final level of the stem weight-gradient reduction, writing only the real taps: the slabs hold
// the stem's padded (OC, 8, 8, 4) layout; dw is the (OC, R, S, IC) gradient (KRSC) in the flat
// buffer. Sums the splits in order (the same fp32 result as wgrad_reduce followed by a strided copy,
// minus that copy's launch).
__global__ void wgrad_reduce_gather_kernel(const float* __restrict__ ws, float* __restrict__ dw, int OC, int R, int S,
                                           int IC, int nsplit, long long slab, float scale, int accumulate) {
  const int n = OC * R * S * IC;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int oc = i / (R * S * IC), rem = i - oc * (R * S * IC);
    const int r = rem / (S * IC), rem2 = rem - r * (S * IC);
    const int s = rem2 / IC, c = rem2 - s * IC;
    const long long src = (long long)oc * 256 + (r * 8 + s) * 4 + c;
    float v = sum_slabs_in_order(ws[src], 1, nsplit, [&](int k) { return ws[(long long)k * slab + src]; });
    v *= scale;
    if (accumulate) v += dw[i];
    dw[i] = v;
  }
}

}  // namespace dbx

using namespace dbx;

int dbx_dispatch_dgrad(int bm, int bn, const IGemmArgs& a, bool accum, int epi, int dma, hipStream_t st);  // conv_dgrad.hip
extern "C" int dbx_conv_patch3(int mode, const IGemmArgs* args, int pro, int stats, int epi, hipStream_t st,
                               int streamed);
extern "C" int dbx_stem_patch(const IGemmArgs* args, int stats, hipStream_t st);

template <int BM, int BN>
static int dispatch_fwd(const IGemmArgs& a, bool pro, bool stats, int dma, hipStream_t st) {
  if (a.res) {
    // 128 x 256 runs as itself: the half-split tail prologue fits it in 256 VGPRs without spills (it
    // was remapped to the same-area 256 x 128 before: one N tile covers a 256-channel conv1, so the
    // shortcut / BN3 operands are read and transformed once instead of twice)
    constexpr int TM = BM, TN = BN;
    if (stats) DBX_DMA_PRO(launch_igemm_t, TM, TN, FWD, true, true, false, 0, true);
    DBX_DMA_PRO(launch_igemm_t, TM, TN, FWD, true, false, false, 0, true);
  }
  if (pro) {
    if (stats) DBX_DMA_PRO(launch_igemm_t, BM, BN, FWD, true, true, false, 0, false);
    DBX_DMA_PRO(launch_igemm_t, BM, BN, FWD, true, false, false, 0, false);
  }
  if (stats) DBX_DMA_PLAIN(launch_igemm_t, BM, BN, FWD, false, true, false, 0, false);
  DBX_DMA_PLAIN(launch_igemm_t, BM, BN, FWD, false, false, false, 0, false);
}


extern "C" int dbx_conv_fast(int mode, int bn, const IGemmArgs* args, int stats, int accum, int epi, hipStream_t st);
extern "C" int dbx_conv_sweep(int mode, const IGemmArgs* args, int pro, int stats, int accum, int epi, hipStream_t st);

extern "C" int dbx_conv_igemm(int mode, int bm, int bn, const IGemmArgs* args, int pro, int stats,
                              int accum, int epi, hipStream_t st, int dma) {
  const IGemmArgs& a = *args;
  if (a.ksplit > 1) {  // split-K: the implicit-GEMM kernel only, every slice non-empty, a counter per tile
    if ((dma != 0 && dma != 1) || mode == STEM || mode == FWD_PATCH || mode == DGRAD_PATCH) return -67;
    if (a.kper < 1 || a.skws == nullptr || a.skcnt == nullptr) return -68;
  }
  if (dma == 8) return dbx_conv_sweep(mode, args, pro, stats, accum, epi, st);  // conv_sweep.hip
  if (dma == 4) {  // eight-wave 256-row kernel (conv_fast.hip): plain operands, stride-1 data gradients
    if (bm != 256 || pro || mode == STEM || (mode == DGRAD && (a.osub != 1 || a.add_sub > 1))) return -65;
    return dbx_conv_fast(mode, bn, args, stats, accum, epi, st);
  }
  if (mode == FWD_PATCH || mode == DGRAD_PATCH) {  // 3x3 weights-stationary patch kernel (conv_patch3.hip)
    if (pro && !a.relu_in) return -7;
    return dbx_conv_patch3(mode == FWD_PATCH ? FWD : DGRAD, args, pro, stats, epi, st, dma);  // dma: 1 = streamed
  }
  if (pro && mode == FWD && !a.relu_in) return -7;  // the forward BN prologue always ends in ReLU
  if (pro && a.IC > (a.res ? 1024 : 512)) return -8;  // prologue coefficients staged in LDS (PRO_MAXC)
  if (a.res && (!pro || mode == STEM || a.R != 1 || a.S != 1 || a.stride != 1 || a.pad != 0))
    return -10;  // the tail prologue is for 1x1 stride-1 consumers (output pixel == input pixel)
  if (a.res && mode == DGRAD && a.tail_bits) return -10;
  if (a.a_out && (mode != DGRAD || epi != 2)) return -9;  // write-back: the MASK_Y epilogue computes it
  if (a.OC % bn != 0) return -1;
  if (mode == STEM) {
    if (pro || accum || epi) return -2;
    if (bm == 0) return dbx_stem_patch(args, stats, st);  // conv_patch3.hip
    if (bm == 128 && bn == 64) return stats ? launch_igemm_t<128, 64, STEM, false, true, false, 0>(a, st)
                                            : launch_igemm_t<128, 64, STEM, false, false, false, 0>(a, st);
    return -3;
  }
  if (a.IC % 64 != 0) return -4;
  if (mode == FWD) {
    if (accum || epi) return -2;
    DBX_TILES(dispatch_fwd, a, pro, stats, dma, st)
    return -3;
  }
  if (mode == DGRAD) {
    if ((pro && !a.res) || stats) return -2;
    if (epi && (a.ybn == nullptr || a.bstats1 == nullptr || a.mean1 == nullptr || a.inv1 == nullptr)) return -6;
    if (epi == 1 && a.mbits == nullptr) return -6;
    if (epi == 2 && (a.bsc == nullptr || a.bsh == nullptr)) return -6;
    return dbx_dispatch_dgrad(bm, bn, a, accum, epi, dma, st);
  }
  return -5;
}

template <int BM, int BN, bool PRO>
static void launch_wgrad_t(const WgradArgs& a, int nblk, hipStream_t st, unsigned lds_pad) {
  // 256-wide tiles on 8 waves (4x2 / 2x4), the rest on 2x2 waves
  constexpr int WM = (BM == 256) ? 4 : 2;
  constexpr int WN = (BN == 256) ? 4 : 2;
  // 8-wave tiles with the BN prologue: one register staging set (two spill at the 256-VGPR cap)
  constexpr int DEPTH = (PRO && (BM == 256 || BN == 256)) ? 1 : 2;
  hipLaunchKernelGGL((wgrad_kernel<BM, BN, WM, WN, FWD, PRO, DEPTH>), dim3(nblk), dim3(64 * WM * WN), lds_pad, st, a);
}

// dma: 2 / 3 = 64-pixel stages in a 2- / 3-slot ring; 4 = 32-pixel stages in a 4-slot ring (the
// 256 x 256 tile's deep ring in 128 KiB)
template <int BM, int BN>
static void launch_wgrad_dma_t(const WgradArgs& a, int nblk, hipStream_t st, unsigned lds_pad, int dma) {
  constexpr bool BIG = BM == 256 && BN == 256;  // 2 x 4 waves of 128 x 64
  constexpr int WM = BIG ? 2 : (BM == 256) ? 4 : 2;
  constexpr int WN = (BN == 256) ? 4 : 2;
  if constexpr (BIG) {
    // (a 5-slot ring of 32-pixel stages measured not faster: profiles/r5_ring/)
    if (dma == 4)
      hipLaunchKernelGGL((wgrad_dma_kernel<BM, BN, WM, WN, 4, 32>), dim3(nblk), dim3(64 * WM * WN), lds_pad, st, a);
    else
      hipLaunchKernelGGL((wgrad_dma_kernel<BM, BN, WM, WN, 2, 64>), dim3(nblk), dim3(64 * WM * WN), lds_pad, st, a);
  } else {
    if (dma == 2)
      hipLaunchKernelGGL((wgrad_dma_kernel<BM, BN, WM, WN, 2>), dim3(nblk), dim3(64 * WM * WN), lds_pad, st, a);
    else
      hipLaunchKernelGGL((wgrad_dma_kernel<BM, BN, WM, WN, 3>), dim3(nblk), dim3(64 * WM * WN), lds_pad, st, a);
  }
}

// lds_pad: extra dynamic LDS per workgroup (bytes) -- an occupancy cap, so that a weight gradient
// running on the side stream leaves room on each CU for the main stream's memory-bound kernels
extern "C" int dbx_conv_wgrad(int mode, int bm, int bn, const WgradArgs* args, int pro, hipStream_t st,
                              unsigned lds_pad, int dma_req) {
  const WgradArgs& a = *args;
  if (pro && !a.relu_in) return -7;  // the BN prologue always ends in ReLU (ResNet dataflow)
  if (a.OC % bm != 0 || a.KTOT % bn != 0) return -1;
  const int nblk = (a.OC / bm) * (a.KTOT / bn) * a.nsplit;
  if (mode == STEM) {
    if (bm == 64 && bn == 128) hipLaunchKernelGGL((wgrad_kernel<64, 128, 2, 2, STEM, false>), dim3(nblk), dim3(256), 0, st, a);
    else return -3;
    return (int)hipGetLastError();
  }
  if (a.IC % bn != 0) return -4;  // a column tile must stay inside one tap
  // LDS-DMA operand path for the prologue-free weight gradients: ring depth 2 or 3, 0 = the
  // register-staged wgrad_kernel; dma_req < 0 = auto: 3 slots for the 8-wave 256-wide tiles (one
  // workgroup per CU either way), 2 for the 4-wave tiles (keeps two workgroups per CU)
  const int dreq = dma_req >= 0 ? dma_req : (bm == 256 && bn == 256) ? 4 : ((bm == 256 || bn == 256) ? 3 : 2);
  int dma = (dreq == 2 || dreq == 3 || dreq == 4) ? dreq : 0;
  if (bm == 256 && bn == 256) {
    if (pro) return -3;      // the 256 x 256 tile is LDS-DMA only (no register-staged prologue variant)
    if (dma == 0) dma = 4;
  } else if (dma == 4) {
    dma = 3;
  }
#define WG(BM_, BN_)                                                                             \
  if (bm == BM_ && bn == BN_) {                                                                  \
    if (pro) launch_wgrad_t<BM_, BN_, true>(a, nblk, st, lds_pad);                               \
    else if (dma) launch_wgrad_dma_t<BM_, BN_>(a, nblk, st, lds_pad, dma);                       \
    else launch_wgrad_t<BM_, BN_, false>(a, nblk, st, lds_pad);                                  \
    return (int)hipGetLastError();                                                               \
  }
  WG(128, 128)
  WG(128, 64)
  WG(64, 128)
  WG(64, 64)
  WG(256, 128)
  WG(128, 256)
  if (bm == 256 && bn == 256) {
    launch_wgrad_dma_t<256, 256>(a, nblk, st, lds_pad, dma);
    return (int)hipGetLastError();
  }
#undef WG
  return -3;
}

// stem: reduce the (OC, 256) slabs into the (OC, R, S, IC) gradient (level 1 as dbx_wgrad_reduce)
extern "C" int dbx_wgrad_reduce_gather(const float* ws, float* dw, int OC, int R, int S, int IC, int nsplit,
                                       float scale, int accumulate, hipStream_t st) {
  if (R > 8 || S > 8 || IC > 4) return -1;
  const long long n = (long long)OC * 256;
  const int n4 = (int)(n / 4);
  const int gx = (n4 + 255) / 256;
  const float* src = ws;
  int parts = nsplit;
  if (nsplit > 8 && (long long)gx * 4 < 1024) {
    int G = 1024 / gx;
    if (G > nsplit / 4) G = nsplit / 4;
    if (G > 64) G = 64;
    if (G < 2) G = 2;
    const int spg = (nsplit + G - 1) / G;
    G = (nsplit + spg - 1) / spg;
    float* ws2 = const_cast<float*>(ws) + (size_t)nsplit * n;
    hipLaunchKernelGGL(wgrad_reduce_l1_kernel, dim3(gx, G), dim3(256), 0, st, ws, ws2, n4, nsplit, spg);
    src = ws2;
    parts = G;
  }
  const int nout = OC * R * S * IC;
  hipLaunchKernelGGL(wgrad_reduce_gather_kernel, dim3((nout + 255) / 256), dim3(256), 0, st, src, dw, OC, R, S, IC,
                     parts, n, scale, accumulate);
  return (int)hipGetLastError();
}

// Batched split-K reductions (the deferred weight-gradient reductions of one side-stream batch): a
// device job table, built once per batch shape (ops/kernels.py ReduceBatch), drives two launches --
// A: level 1 of every two-level job (the same groups as dbx_wgrad_reduce), B: every job's final sum;
// per element the same adds in the same order as the per-gradient reduce, so the gradients are
// bit-identical; two launches per batch instead of one or two per weight gradient. Each workgroup
// serves ONE job (a block range per job): it finds the job from blockIdx alone and reads the job
// once, uniformly, before its loop. (A per-lane lookup in a by-value job table gave run-to-run
// different results inside replayed graphs, and big by-value tables in many graph nodes are avoided
// altogether: profiles/r4_s10/, r4_s12/.)
struct RJob {
  const float* ws;    // nsplit slabs of n floats (+ the level-1 partials after them)
  float* dw;
  int n4, nsplit, G, spg, accumulate;
  float scale;
  int bA, bB;         // first workgroup of the job in launch A (two-level jobs, else -1) / launch B
};
__device__ __forceinline__ int rjob_find(const RJob* __restrict__ J, int nj, bool levA) {
  const int b = (int)blockIdx.x;
  int k = -1;
  for (int q = 0; q < nj; ++q) {  // (uniform: every lane scans the same table)
    const int s = levA ? J[q].bA : J[q].bB;
    if (s >= 0 && s <= b) k = q;
  }
  return __builtin_amdgcn_readfirstlane(k);
}
__global__ void wgrad_reduce_multi_l1_kernel(const RJob* __restrict__ J, int nj, int nblocks) {
  const int k = rjob_find(J, nj, true);
  const RJob r = J[k];
  int nb = nblocks - r.bA;  // blocks of this job: up to the next two-level job's first block
  for (int q = k + 1; q < nj; ++q)
    if (J[q].bA >= 0) { nb = J[q].bA - r.bA; break; }
  const f32x4* w4 = reinterpret_cast<const f32x4*>(r.ws);
  f32x4* p4 = reinterpret_cast<f32x4*>(const_cast<float*>(r.ws) + (size_t)r.nsplit * r.n4 * 4);
  const long long items = (long long)r.G * r.n4;
  for (long long f = (long long)((int)blockIdx.x - r.bA) * blockDim.x + threadIdx.x; f < items;
       f += (long long)nb * blockDim.x) {
    const int g = (int)(f / r.n4), i = (int)(f - (long long)g * r.n4);
    const int s0 = g * r.spg, s1 = min(r.nsplit, s0 + r.spg);
    p4[(size_t)g * r.n4 + i] = sum_slabs_in_order(f32x4{0.f, 0.f, 0.f, 0.f}, s0, s1,
                                                  [&](int kk) { return w4[(size_t)kk * r.n4 + i]; });
  }
}
__global__ void wgrad_reduce_multi_kernel(const RJob* __restrict__ J, int nj, int nblocks) {
  const int k = rjob_find(J, nj, false);
  const RJob r = J[k];
  const int nb = (k + 1 < nj ? J[k + 1].bB : nblocks) - r.bB;
  // two-level jobs sum their G group partials, single-level ones their nsplit slabs
  const f32x4* w4 = reinterpret_cast<const f32x4*>(r.G > 1 ? r.ws + (size_t)r.nsplit * r.n4 * 4 : r.ws);
  const int cnt = r.G > 1 ? r.G : r.nsplit;
  f32x4* o4 = reinterpret_cast<f32x4*>(r.dw);
  for (int i = ((int)blockIdx.x - r.bB) * blockDim.x + threadIdx.x; i < r.n4; i += nb * blockDim.x) {
    f32x4 sm = sum_slabs_in_order(w4[i], 1, cnt, [&](int kk) { return w4[(size_t)kk * r.n4 + i]; });
    sm *= r.scale;
    if (r.accumulate) sm += o4[i];
    o4[i] = sm;
  }
}

// Host side of the job table: fills `table` (host memory, njobs RJob entries) from the job lists and
// returns the two grid sizes; the caller copies the table to the device once per batch shape.
extern "C" int dbx_wgrad_reduce_multi_plan(const float* const* ws, float* const* dw, const long long* n,
                                           const int* nsplit, const float* scale, const int* accumulate, int njobs,
                                           void* table, int* grid_a, int* grid_b) {
  auto blocks_for = [](long long items) {
    const long long b = (items + 255) / 256;
    return (int)(b < 1 ? 1 : (b > 1024 ? 1024 : b));
  };
  RJob* T = reinterpret_cast<RJob*>(table);
  int ga = 0, gb = 0;
  for (int q = 0; q < njobs; ++q) {
    if (n[q] % 4) return -1;
    RJob r{ws[q], dw[q], (int)(n[q] / 4), nsplit[q], 1, 1, accumulate[q], scale[q], -1, gb};
    const int gx = (r.n4 + 255) / 256;
    if (r.nsplit > 8 && (long long)gx * 4 < 1024) {
      int G = 1024 / gx;
      if (G > r.nsplit / 4) G = r.nsplit / 4;
      if (G > 64) G = 64;
      if (G < 2) G = 2;
      r.spg = (r.nsplit + G - 1) / G;
      r.G = (r.nsplit + r.spg - 1) / r.spg;
      r.bA = ga;
      ga += blocks_for((long long)r.G * r.n4);
    }
    gb += blocks_for(r.n4);
    T[q] = r;
  }
  *grid_a = ga;
  *grid_b = gb;
  return 0;
}
extern "C" int dbx_wgrad_reduce_multi_run(const void* table_dev, int njobs, int grid_a, int grid_b, hipStream_t st) {
  const RJob* J = reinterpret_cast<const RJob*>(table_dev);
  if (grid_a > 0) hipLaunchKernelGGL(wgrad_reduce_multi_l1_kernel, dim3(grid_a), dim3(256), 0, st, J, njobs, grid_a);
  hipLaunchKernelGGL(wgrad_reduce_multi_kernel, dim3(grid_b), dim3(256), 0, st, J, njobs, grid_b);
  return (int)hipGetLastError();
}
extern "C" int dbx_wgrad_reduce_job_bytes() { return (int)sizeof(RJob); }

extern "C" int dbx_wgrad_reduce(const float* ws, float* dw, long long n, int nsplit, float scale,
                                int accumulate, hipStream_t st) {
  if (n % 4) return -1;
  const int n4 = (int)(n / 4);
  const int gx = (n4 + 255) / 256;
  if (nsplit > 8 && (long long)gx * 4 < 1024) {
    // level 1 into the tail of the workspace (after the nsplit slabs)
    int G = 1024 / gx;
    if (G > nsplit / 4) G = nsplit / 4;
    if (G > 64) G = 64;
    if (G < 2) G = 2;
    const int spg = (nsplit + G - 1) / G;
    G = (nsplit + spg - 1) / spg;
    float* ws2 = const_cast<float*>(ws) + (size_t)nsplit * n;
    hipLaunchKernelGGL(wgrad_reduce_l1_kernel, dim3(gx, G), dim3(256), 0, st, ws, ws2, n4, nsplit, spg);
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(gx), dim3(256), 0, st, ws2, dw, n4, G, scale, accumulate);
  } else {
    const int grid = gx > 4096 ? 4096 : gx;
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(grid), dim3(256), 0, st, ws, dw, n4, nsplit, scale, accumulate);
  }
  return (int)hipGetLastError();
}
