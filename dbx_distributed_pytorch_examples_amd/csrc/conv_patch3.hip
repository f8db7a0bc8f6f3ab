// 3x3 stride-1 convolutions of the 64-channel ResNet stage as a weights-stationary "patch" kernel.
//
// The implicit-GEMM kernel (conv_igemm_kernel.h) stages one (pixel x 64-channel) block of A per
// filter tap, so every input element is gathered, BN-transformed (forward prologue) and written to
// LDS nine times. For the 64 -> 64 3x3 convs at 56x56 (N = 64: little MFMA work per staged byte)
// that made them VALU- and latency-bound at ~18 % MFMA (profiles/r2s3_patch/). Here a workgroup
// owns TR full output rows of one image (BM = TR * W pixels) and
//   * keeps ALL 9 x 64 x 64 weights resident in LDS (loaded once per workgroup: persistent grid),
//   * stages the input patch (TR + 2 rows x W + 2 columns x 64 channels, halo zero-filled) ONCE
//     per tile, applying the BN prologue once per element,
//   * runs the 9 taps straight out of the patch (tap = an address offset; no barrier inside the
//     K loop), the next tile's patch loads in flight in registers meanwhile,
//   * finishes with the shared igemm epilogue (BN statistics / BN-backward MASK_Y epilogue).
// FWD:   Y[n,h,w,k]  = sum_{r,s,c} act(X[n,h-1+r,w-1+s,c]) W[k][r][s][c]
// DGRAD: dX[n,h,w,c] = sum_{r,s,k} dY[n,h+1-r,w+1-s,k] Wt[c][r][s][k]     (3x3, pad 1, stride 1)
// Weight rows use the conv kernels' XOR swizzle (chunk ^ ((row >> 1) & 7)). The patch swizzle is a
// function of the OUTPUT-linear index x = p - 2 * (p / PC) (= q + dr*W + ds for the pixel a tap reads):
// chunk ^ (x & 6). A tap shifts the 16 pixels of a fragment by an arbitrary (often odd) amount, and
// (x & 6) is the swizzle under which every lane group of a ds_read_b128 fragment read hits 16
// distinct 16-byte bank groups for every shift (found by exhaustive search over the gfx950 lane
// groups; the row swizzle (x >> 1) & 7 gave 2-way conflicts on odd shifts).
#include "conv_igemm_kernel.h"

namespace dbx {

template <int MODE, bool PRO, bool STATS, int EPI, int TR, int WIDTH>
__global__ __launch_bounds__(512, 1) void patch3_kernel(const IGemmArgs a) {
  constexpr int C = 64, BN = 64;          // input / output channels of the patch convs
  constexpr int WM = 4, WN = 2, NT = 512;  // 8 waves: each (BM/4) pixels x 32 channels
  constexpr int BM = TR * WIDTH;
  constexpr int TM = BM / (16 * WM), TN = BN / (16 * WN);
  static_assert(BM % (16 * WM) == 0, "tile rows must split into 16-row MFMA blocks per wave");
  constexpr int PC = WIDTH + 2, PR = TR + 2, PPIX = PR * PC;
  constexpr int PCH = PPIX * 8;               // 16-byte chunks of one patch image
  constexpr int PU = (PCH + NT - 1) / NT;     // patch chunks per thread
  constexpr int WCH = 9 * BN * 8;             // weight chunks (9 taps x 64 rows x 8)
  static_assert(WCH % NT == 0, "weight staging");
  constexpr int LDS_W = 9 * BN * C;           // bf16 elements
  constexpr int LDS_P = PPIX * C;
  static_assert(LDS_P >= BM * (BN + 8), "the epilogue stages its tile through the patch image");
  __shared__ __attribute__((aligned(16))) bf16 lds[LDS_W + LDS_P];
  bf16* sW = lds;
  bf16* sP = lds + LDS_W;
  __shared__ float sPro[2 * C];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wm = wid / WN, wn = wid % WN;
  const int H = a.OH;  // stride 1, pad 1: output rows == input rows
  const int ntile = a.N * H / TR;

  // ---- resident weights: B[tap][n][k] (FWD: W[n][tap*64 + k]; DGRAD: Wt[n][tap*64 + k]) --------
#pragma unroll
  for (int u = 0; u < WCH / NT; ++u) {
    const int e = tid + NT * u;           // chunk: (tap, row n, chunk ch)
    const int ch = e & 7, n = (e >> 3) & 63, tap = e >> 9;
    const u32x4 v = *reinterpret_cast<const u32x4*>(a.w + (size_t)n * (9 * C) + tap * C + ch * 8);
    *reinterpret_cast<u32x4*>(sW + tap * BN * C + n * C + ((ch ^ ((n >> 1) & 7)) << 3)) = v;
  }
  if constexpr (PRO) {
    for (int c = tid; c < C; c += NT) { sPro[c] = a.in_scale[c]; sPro[C + c] = a.in_shift[c]; }
  }

  // ---- patch staging: chunk e = tid + NT*u -> patch pixel p = e / 8 (row p / PC, col p % PC) -------
  const rsrc_t xr = make_rsrc(a.x, 2ull * a.N * H * WIDTH * C);
  u32x4 pv[PU];
  unsigned pval = 0;  // bit u: chunk u is an in-image pixel (padding stays exactly zero after PRO)
  auto load_patch = [&](int t) __attribute__((always_inline)) {
    const int g0 = t * TR, n = g0 / H, h0 = g0 - n * H;
    pval = 0;
#pragma unroll
    for (int u = 0; u < PU; ++u) {
      const int e = tid + NT * u;
      const int p = e >> 3, ch = e & 7;
      const int pr = p / PC, pc = p - pr * PC;
      const int h = h0 - 1 + pr, w = pc - 1;
      const bool v = e < PCH && t < ntile && (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)WIDTH;
      pv[u] = buf_load16(xr, v ? 2u * (unsigned)((((n * H + h) * WIDTH) + w) * C + ch * 8) : kOOB);
      pval |= (v ? 1u : 0u) << u;
    }
  };
  auto store_patch = [&]() __attribute__((always_inline)) {
    // this thread's 8 channels are the same for every chunk (NT % 8 == 0): coefficients read once
    f32x4 s0, s1, h0, h1;
    if constexpr (PRO) {
      s0 = *reinterpret_cast<const f32x4*>(sPro + (tid & 7) * 8);
      s1 = *reinterpret_cast<const f32x4*>(sPro + (tid & 7) * 8 + 4);
      h0 = *reinterpret_cast<const f32x4*>(sPro + C + (tid & 7) * 8);
      h1 = *reinterpret_cast<const f32x4*>(sPro + C + (tid & 7) * 8 + 4);
    }
#pragma unroll
    for (int u = 0; u < PU; ++u) {
      const int e = tid + NT * u;
      if (PCH % NT != 0 && e >= PCH) break;  // (only the last chunk set can be partial)
      const int p = e >> 3, ch = e & 7;
      u32x4 v = pv[u];
      if constexpr (PRO) {
        float f[8];
        unpack8(v, f);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          f[j] = f[j] * s0[j] + h0[j];
          f[j + 4] = f[j + 4] * s1[j] + h1[j];
        }
        const u32x4 z = {0u, 0u, 0u, 0u};
        v = ((pval >> u) & 1u) ? relu_bf16x8(pack8(f)) : z;
      }
      const int x = p - 2 * (p / PC);
      *reinterpret_cast<u32x4*>(sP + p * C + ((ch ^ (x & 6)) << 3)) = v;
    }
  };

  // ---- per-lane fragment geometry ------------------------------------------------------------
  // A: output pixel q = wm*(BM/WM) + i*16 + (lane & 15) of the tile -> patch pixel of tap (0, 0)
  int pbase[TM], qbase[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int q = wm * (BM / WM) + i * 16 + (lane & 15);
    const int oi = q / WIDTH, oj = q - oi * WIDTH;
    pbase[i] = oi * PC + oj;
    qbase[i] = q;
  }
  const int kq = lane >> 4;  // chunk within a 32-wide K step: ks*4 + kq

  int t = blockIdx.x;
  load_patch(t);
  __syncthreads();  // sPro
  store_patch();
  f32x4 acc[TM][TN];
  for (;;) {
    __syncthreads();  // patch(t) (and on the first tile the weights) visible
    const int tn = t + gridDim.x;
    if (tn < ntile) load_patch(tn);  // in flight during the MFMAs (workgroup-uniform branch)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // Fragment reads are software-pipelined one half-tap ahead (two register sets: the reads of
    // step k+1 are in flight while step k's 14 MFMAs issue). Taps are not unrolled: per-tap
    // fragment addresses are computed in the loop instead of being hoisted out of the persistent
    // loop by the compiler (7 x 9 x 2 live addresses would spill).
    bf16x8 afA[TM], bfA[TN], afB[TM], bfB[TN];
    auto frags = [&](int tap, int ks, bf16x8 (&af)[TM], bf16x8 (&bf)[TN]) __attribute__((always_inline)) {
      const int r = tap / 3, s = tap - 3 * r;
      // FWD reads input (h - 1 + r, w - 1 + s) = patch (oi + r, oj + s); DGRAD reads dY at
      // (h + 1 - r, w + 1 - s) = patch (oi + 2 - r, oj + 2 - s)
      const int dr = (MODE == DGRAD) ? 2 - r : r, ds = (MODE == DGRAD) ? 2 - s : s;
      const int doff = dr * PC + ds, dx = dr * WIDTH + ds;
      const int ch = ks * 4 + kq;
      const bf16* cB = sW + tap * BN * C;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * (BN / WN) + j * 16 + (lane & 15);
        bf[j] = *reinterpret_cast<const bf16x8*>(cB + row * C + ((ch ^ ((row >> 1) & 7)) << 3));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int p = pbase[i] + doff, x = qbase[i] + dx;
        af[i] = *reinterpret_cast<const bf16x8*>(sP + p * C + ((ch ^ (x & 6)) << 3));
      }
    };
    auto mma = [&](const bf16x8 (&af)[TM], const bf16x8 (&bf)[TN]) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j], af[i], acc[i][j], 0, 0, 0);
    };
    frags(0, 0, afA, bfA);
#pragma unroll 1
    for (int tap = 0; tap < 9; ++tap) {
      frags(tap, 1, afB, bfB);
      mma(afA, bfA);
      frags(tap < 8 ? tap + 1 : 8, 0, afA, bfA);  // (past the last tap: a harmless re-read)
      mma(afB, bfB);
    }
    __syncthreads();  // every wave is done with patch(t): the epilogue stages through it
    // (row groups of 2 in the BN-backward epilogue: the next patch's registers stay live across it)
    igemm_epilogue<BM, BN, WM, WN, MODE, STATS, false, EPI, (EPI ? 2 : 4)>(a, acc, sP, t * BM, 0, t, blockIdx.x);
    if (tn >= ntile) break;
    __syncthreads();  // the epilogue's LDS reads are done
    store_patch();
    t = tn;
  }
}


// Streamed-weights variant: 4 waves, one tile of TR rows per workgroup (not persistent), the patch
// by LDS-DMA (no prologue) or register-staged (BN prologue), the 9 per-tap weight blocks by
// LDS-DMA through a 3-slot ring. ~68 KB of LDS instead of ~148 KB: two workgroups share a CU, so
// one's epilogue (the BN-backward MASK_Y epilogue streams three tensors) overlaps the other's MFMAs
// -- which the single resident-weights workgroup per CU cannot do.
template <int MODE, bool PRO, bool STATS, int EPI, int TR, int WIDTH>
__global__ __launch_bounds__(256, 2) void patch3s_kernel(const IGemmArgs a) {
  constexpr int C = 64, BN = 64;
  constexpr int WM = 2, WN = 2, NT = 256, NW = 4;
  constexpr int BM = TR * WIDTH;
  constexpr int TM = BM / (16 * WM), TN = BN / (16 * WN);
  static_assert(BM % (16 * WM) == 0, "tile rows must split into 16-row MFMA blocks per wave");
  constexpr int PC = WIDTH + 2, PR = TR + 2, PPIX = PR * PC;
  constexpr int PCH = PPIX * 8;                      // 16-byte chunks of the patch image
  constexpr int PDI = (PCH + 64 * NW - 1) / (64 * NW);  // patch DMA instructions per wave
  constexpr int LDS_P = PDI * NW * 64 * 8;           // bf16 elements (whole 1 KiB DMA pieces)
  constexpr int NB = 3;                              // weight ring slots
  constexpr int WSLOT = BN * C;                      // one tap's weights
  static_assert(LDS_P >= BM * (BN + 8), "the epilogue stages its tile through the patch image");
  __shared__ __attribute__((aligned(1024))) bf16 lds[LDS_P + NB * WSLOT];
  bf16* sP = lds;
  bf16* sW = lds + LDS_P;
  __shared__ float sPro[2 * C];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wm = wid / WN, wn = wid % WN;
  const int H = a.OH;
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int g0 = t * TR, n = g0 / H, h0 = g0 - n * H;
  const unsigned lbase = lds_addr(lds);
  const i32x4 wsrd = make_srd(a.w, 2ull * BN * 9 * C);

  // weights of tap k -> ring slot k % NB: lane fills row wr = 8*(wid + NW*i) + lane/8, slot lane%8
  // with source chunk slot ^ ((row >> 1) & 7) (the row swizzle, inverted at the source)
  auto dma_w = [&](int tap) __attribute__((always_inline)) {
    const unsigned dst = lbase + 2u * (unsigned)(LDS_P + (tap % NB) * WSLOT) + 1024u * (unsigned)wid;
#pragma unroll
    for (int i = 0; i < WSLOT / 8 / (64 * NW); ++i) {
      const int row = 8 * (wid + NW * i) + (lane >> 3);
      const int src = (lane & 7) ^ ((row >> 1) & 7);
      const unsigned off = tap < 9 ? 2u * (unsigned)(row * 9 * C + tap * C + src * 8) : kOOB;
      lds_dma16(wsrd, off, dst + 1024u * (unsigned)(NW * i));
    }
  };
  constexpr int WDI = WSLOT / 8 / (64 * NW);  // weight DMA instructions per wave and tap

  // ---- patch ------------------------------------------------------------------------------
  if constexpr (!PRO) {
    const i32x4 xsrd = make_srd(a.x, 2ull * a.N * H * WIDTH * C);
#pragma unroll
    for (int i = 0; i < PDI; ++i) {
      const int e = 64 * (wid + NW * i) + lane;  // LDS chunk position
      const int p = e >> 3;
      const int pr = p / PC, pc = p - pr * PC;
      const int x = p - 2 * pr;
      const int ch = (lane & 7) ^ (x & 6);
      const int h = h0 - 1 + pr, w = pc - 1;
      const bool v = e < PCH && (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)WIDTH;
      lds_dma16(xsrd, v ? 2u * (unsigned)((((n * H + h) * WIDTH) + w) * C + ch * 8) : kOOB,
                lbase + 1024u * (unsigned)(wid + NW * i));
    }
    dma_w(0);
    dma_w(1);
  } else {
    dma_w(0);
    dma_w(1);
    for (int c = tid; c < C; c += NT) { sPro[c] = a.in_scale[c]; sPro[C + c] = a.in_shift[c]; }
    __syncthreads();
    const rsrc_t xr = make_rsrc(a.x, 2ull * a.N * H * WIDTH * C);
    const f32x4 s0 = *reinterpret_cast<const f32x4*>(sPro + (tid & 7) * 8);
    const f32x4 s1 = *reinterpret_cast<const f32x4*>(sPro + (tid & 7) * 8 + 4);
    const f32x4 f0 = *reinterpret_cast<const f32x4*>(sPro + C + (tid & 7) * 8);
    const f32x4 f1 = *reinterpret_cast<const f32x4*>(sPro + C + (tid & 7) * 8 + 4);
    constexpr int PU = (PCH + NT - 1) / NT;
    u32x4 pv[PU];
    unsigned pval = 0;
#pragma unroll
    for (int u = 0; u < PU; ++u) {
      const int e = tid + NT * u;
      const int p = e >> 3, ch = e & 7;
      const int pr = p / PC, pc = p - pr * PC;
      const int h = h0 - 1 + pr, w = pc - 1;
      const bool v = e < PCH && (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)WIDTH;
      pv[u] = buf_load16(xr, v ? 2u * (unsigned)((((n * H + h) * WIDTH) + w) * C + ch * 8) : kOOB);
      pval |= (v ? 1u : 0u) << u;
    }
#pragma unroll
    for (int u = 0; u < PU; ++u) {
      const int e = tid + NT * u;
      if (PCH % NT != 0 && e >= PCH) break;
      const int p = e >> 3, ch = e & 7;
      float f[8];
      unpack8(pv[u], f);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        f[j] = f[j] * s0[j] + f0[j];
        f[j + 4] = f[j + 4] * s1[j] + f1[j];
      }
      const u32x4 z = {0u, 0u, 0u, 0u};
      const int x = p - 2 * (p / PC);
      *reinterpret_cast<u32x4*>(sP + p * C + ((ch ^ (x & 6)) << 3)) = ((pval >> u) & 1u) ? relu_bf16x8(pack8(f)) : z;
    }
  }

  // ---- MFMAs: 9 taps out of the patch, weights through the ring -----------------------------
  int pbase[TM], qbase[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int q = wm * (BM / WM) + i * 16 + (lane & 15);
    const int oi = q / WIDTH, oj = q - oi * WIDTH;
    pbase[i] = oi * PC + oj;
    qbase[i] = q;
  }
  const int kq = lane >> 4;
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
  for (int tap = 0; tap < 9; ++tap) {
    // this wave's share of tap's weights (and, at tap 0, of the patch) has landed; the barrier
    // publishes every wave's and retires the slot the next issue overwrites
    dma_wait<WDI>();
    __syncthreads();
    dma_w(tap + 2);
    const int r = tap / 3, s = tap - 3 * r;
    const int dr = (MODE == DGRAD) ? 2 - r : r, ds = (MODE == DGRAD) ? 2 - s : s;
    const int doff = dr * PC + ds, dx = dr * WIDTH + ds;
    const bf16* cB = sW + (tap % NB) * WSLOT;
    bf16x8 af[2][TM], bfr[2][TN];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ch = ks * 4 + kq;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * (BN / WN) + j * 16 + (lane & 15);
        bfr[ks][j] = *reinterpret_cast<const bf16x8*>(cB + row * C + ((ch ^ ((row >> 1) & 7)) << 3));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int p = pbase[i] + doff, x = qbase[i] + dx;
        af[ks][i] = *reinterpret_cast<const bf16x8*>(sP + p * C + ((ch ^ (x & 6)) << 3));
      }
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[ks][j], af[ks][i], acc[i][j], 0, 0, 0);
  }
  dma_wait<0>();
  __syncthreads();  // every wave is done with the patch: the epilogue stages through it
  igemm_epilogue<BM, BN, WM, WN, MODE, STATS, false, EPI>(a, acc, sP, t * BM, 0, t, blockIdx.x);
}


// ---------------------------------------------------------------------------------------------
// The 7x7 stride-2 stem on the NHWC4 image as a patch kernel. A tile is TR output rows x 112 (448
// pixels); its input patch (2TR+5 rows x 232 columns x 4 channels, 16-byte chunks = pixel pairs,
// columns -4..227 so a pair never straddles the image border) arrives by LDS-DMA, double-buffered
// (the next tile's patch lands during this tile's MFMAs and epilogue). A K step is one filter row
// r: 8 taps x 4 channels; the weights are shifted by one tap (s' = s + 1, s' = 0 is zero) so that
// every fragment read is one aligned pixel pair: patch chunk (2*oi + r) * 116 + oj + kq. Filter row
// 7 does not exist, so 7 K steps of 32 (224 padded K for 147 real; the implicit GEMM used 256).
// All offsets of a fragment read are immediates off two per-lane bases; no per-step VALU.
template <bool STATS, int TR>
__global__ __launch_bounds__(512, 1) void stem_patch_kernel(const IGemmArgs a) {
  constexpr int OW = 112, IW = 224, BN = 64;
  constexpr int WM = 4, WN = 2, NT = 512, NW = 8;
  constexpr int BM = TR * OW;
  constexpr int TM = BM / (16 * WM), TN = BN / (16 * WN);
  static_assert(BM % (16 * WM) == 0, "tile rows");
  constexpr int PCC = 116;                             // 16-byte chunks per patch row (232 pixels)
  constexpr int PROWS = 2 * TR + 5;
  constexpr int PCH = PROWS * PCC;
  constexpr int PDI = (PCH + 64 * NW - 1) / (64 * NW);  // DMA instructions per wave per patch
  constexpr int PBUF = PDI * NW * 64 * 8;              // bf16 elements per patch buffer
  constexpr int WP = 240;                              // weight row pitch (224 + 16: conflict-free)
  constexpr int LDS_C = BM * (BN + 8);
  __shared__ __attribute__((aligned(1024))) bf16 lds[2 * PBUF + BN * WP + LDS_C];
  bf16* sP = lds;                  // [2][PBUF]
  bf16* sW = lds + 2 * PBUF;       // [64][WP]
  bf16* sC = sW + BN * WP;         // epilogue staging (its own region: the patches stay live)

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wm = wid / WN, wn = wid % WN;
  const int ntile = a.N * (a.OH / TR);
  constexpr int TPI = 112 / TR;  // tiles per image

  // shifted weights: W'[n][r*32 + s'*4 + c] = W[n][r*32 + (s'-1)*4 + c] (s' = 0: zero), r < 7
  for (int e = tid; e < BN * 28; e += NT) {
    const int n = e / 28, q = e - n * 28, r = q >> 2, j = q & 3;  // chunk j of filter row r: s' = 2j, 2j+1
    const bf16* src = a.w + n * 256 + r * 32 + 8 * j;  // taps s = 2j (hi half); s = 2j - 1 (lo half)
    const uint2 hi = *reinterpret_cast<const uint2*>(src);
    uint2 lo = *reinterpret_cast<const uint2*>(src - (j ? 4 : 0));  // (j = 0: an in-range stand-in)
    if (j == 0) lo = uint2{0u, 0u};
    *reinterpret_cast<u32x4*>(sW + n * WP + r * 32 + j * 8) = u32x4{lo.x, lo.y, hi.x, hi.y};
  }

  const i32x4 xsrd = make_srd(a.x, 2ull * a.N * a.IH * IW * 4);
  const unsigned lbase = lds_addr(lds);
  auto dma_patch = [&](int t, int buf) __attribute__((always_inline)) {
    const int n = t / TPI, oh0 = (t - n * TPI) * TR;
    const int ih0 = 2 * oh0 - 3;
#pragma unroll
    for (int i = 0; i < PDI; ++i) {
      const int e = 64 * (wid + NW * i) + lane;
      const int pr = e / PCC, pc = e - pr * PCC;
      const int ih = ih0 + pr, iw = 2 * pc - 4;
      const bool v = e < PCH && (unsigned)ih < (unsigned)a.IH && (unsigned)iw < (unsigned)IW;
      lds_dma16(xsrd, v ? 8u * (unsigned)((n * a.IH + ih) * IW + iw) : kOOB,
                lbase + 2u * (unsigned)(buf * PBUF) + 1024u * (unsigned)(wid + NW * i));
    }
  };

  // per-lane fragment bases (bytes): A = pixel pair of output pixel q at filter row 0, B = row n
  unsigned abase[TM], bbase[TN];
  const int kq = lane >> 4;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int q = wm * (BM / WM) + i * 16 + (lane & 15);
    const int oi = q / OW, oj = q - oi * OW;
    abase[i] = 16u * (unsigned)(2 * oi * PCC + oj + kq);
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) bbase[j] = 2u * (unsigned)((wn * (BN / WN) + j * 16 + (lane & 15)) * WP + kq * 8);

  int t = blockIdx.x;
  dma_patch(t, 0);
  f32x4 acc[TM][TN];
  // vector-memory ops a thread issues after a patch DMA: the epilogue's NIT row stores (and, for the
  // first 64 threads, 2 statistics atomics): waiting for that many younger ops retires the DMA
  constexpr int NST = BM * (BN / 8) / NT;
  for (int it = 0;; ++it) {
    if (it == 0) dma_wait<0>();
    else dma_wait<NST>();
    __syncthreads();  // patch(t) landed for every wave; (first tile) the weights are visible
    const int tn = t + gridDim.x;
    if (tn < ntile) dma_patch(tn, (it + 1) & 1);  // into the buffer tile t-1 read
    const char* cP = reinterpret_cast<const char*>(sP + (it & 1) * PBUF);
    const char* cW = reinterpret_cast<const char*>(sW);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < 7; ++r) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(cW + bbase[j] + 64 * r);
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const bf16x8*>(cP + abase[i] + 16 * PCC * r);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    }
    igemm_epilogue<BM, BN, WM, WN, FWD, STATS, false, 0>(a, acc, sC, t * BM, 0, t, blockIdx.x);
    if (tn >= ntile) break;
    t = tn;
  }
  dma_wait<0>();
}


// ---------------------------------------------------------------------------------------------
// Weight gradient of the 64 -> 64 3x3 stride-1 convs as a patch kernel:
//   dW[k][tap][c] = sum_q dY[q][k] * X[q (+) tap][c]        (X = the stored BN output, zero halo)
// A workgroup (4 waves, one per CU, persistent) walks tiles of TR output rows; per tile the dY rows
// and the (TR+2) x (W+2) input patch arrive by LDS-DMA (double-buffered: the next tile lands during
// this one). Wave w owns channels c = 16w..16w+15 of ALL 9 taps x 64 k (36 accumulator blocks), so
// per 32-pixel K step it reads 4 dY fragments and 9 patch fragments for 36 MFMAs; the tap is a row
// offset into the patch (transposed reads, ds_read_b64_tr_b16). Both images use the wgrad tr_swz
// chunk swizzle keyed on the OUTPUT-linear pixel index (for the patch x = p - 2 * (p / PC)), which
// keeps the shifted transposed reads conflict-free for every tap (exhaustive check over shifts).
// Each workgroup writes one fp32 partial slab of dW; wgrad_reduce sums them in a fixed order.
__device__ __forceinline__ int trx(int x) {  // tr_swz(row, ., 8) XOR term (conv_igemm.hip)
  return ((((x & 1) << 2) ^ (x & 2) ^ (((x >> 3) & 1) << 2)) & 7);
}

template <int TR, int WIDTH>
__global__ __launch_bounds__(256, 1) void wgrad_patch3_kernel(const WgradArgs a) {
  constexpr int C = 64, NW = 4;
  constexpr int BMP = TR * WIDTH;                    // pixels per tile (K of the tile's GEMM)
  static_assert(BMP % 32 == 0, "tile pixels must be whole 32-pixel K steps");
  constexpr int KS = BMP / 32;
  constexpr int PC = WIDTH + 2, PR = TR + 2, PPIX = PR * PC;
  constexpr int DYI = (BMP * 8 + 64 * NW - 1) / (64 * NW);   // dY DMA instructions per wave
  constexpr int PAI = (PPIX * 8 + 64 * NW - 1) / (64 * NW);  // patch DMA instructions per wave
  constexpr int DYE = DYI * NW * 64 * 8, PAE = PAI * NW * 64 * 8;  // bf16 elements per image
  constexpr int BUF = DYE + PAE;
  __shared__ __attribute__((aligned(1024))) bf16 lds[2 * BUF];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int H = a.OH;
  const int ntile = a.N * H / TR;
  const i32x4 dysrd = make_srd(a.dy, 2ull * a.M * C);
  const i32x4 xsrd = make_srd(a.x, 2ull * a.N * H * WIDTH * C);
  const unsigned lbase = lds_addr(lds);

  auto dma_tile = [&](int t, int buf) __attribute__((always_inline)) {
    const int g0 = t * TR, n = g0 / H, h0 = g0 - n * H;
    const unsigned dst = lbase + 2u * (unsigned)(buf * BUF);
#pragma unroll
    for (int i = 0; i < DYI; ++i) {
      const int e = 64 * (wid + NW * i) + lane;
      const int row = e >> 3, src = (lane & 7) ^ trx(row);
      const unsigned off = row < BMP ? 2u * (unsigned)((g0 * WIDTH + row) * C + src * 8) : kOOB;
      lds_dma16(dysrd, off, dst + 1024u * (unsigned)(wid + NW * i));
    }
#pragma unroll
    for (int i = 0; i < PAI; ++i) {
      const int e = 64 * (wid + NW * i) + lane;
      const int pp = e >> 3, pr = pp / PC, pc = pp - pr * PC;
      const int src = (lane & 7) ^ trx(pp - 2 * pr);
      const int h = h0 - 1 + pr, w = pc - 1;
      const bool v = pp < PPIX && (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)WIDTH;
      lds_dma16(xsrd, v ? 2u * (unsigned)(((n * H + h) * WIDTH + w) * C + src * 8) : kOOB,
                dst + 2u * (unsigned)DYE + 1024u * (unsigned)(wid + NW * i));
    }
  };

  f32x4 acc[4][9];
#pragma unroll
  for (int kb = 0; kb < 4; ++kb)
#pragma unroll
    for (int tp = 0; tp < 9; ++tp) acc[kb][tp] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int g = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
  int t = blockIdx.x;
  dma_tile(t, 0);
  for (int it = 0;; ++it) {
    dma_wait<0>();
    __syncthreads();  // tile t landed (every wave's part); the other buffer is no longer read
    const int tn = t + gridDim.x;
    if (tn < ntile) dma_tile(tn, (it + 1) & 1);
    const bf16* cA = lds + (it & 1) * BUF;
    const bf16* cP = cA + DYE;
#pragma unroll 1
    for (int js = 0; js < KS; ++js) {
      s16x4 va[2][4], vb[2][9];  // [lo / hi: pixel rows +0 / +4]
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const int row = js * 32 + 8 * g + q4 + 4 * h2;
        const int oi = row / WIDTH, oj = row - oi * WIDTH;
        const int pp0 = oi * PC + oj;
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) {
          const int col = kb * 16 + 4 * p4;
          va[h2][kb] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (DBX_LDS s16x4*)(cA + row * C + (((col >> 3) ^ trx(row)) << 3) + (col & 7)));
        }
        const int colb = wid * 16 + 4 * p4;
#pragma unroll
        for (int tp = 0; tp < 9; ++tp) {
          const int r = tp / 3, sx = tp - 3 * (tp / 3);
          const int pp = pp0 + r * PC + sx, x = row + r * WIDTH + sx;
          vb[h2][tp] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (DBX_LDS s16x4*)(cP + pp * C + (((colb >> 3) ^ trx(x)) << 3) + (colb & 7)));
        }
      }
      bf16x8 af[4], bfr[9];
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
        af[kb] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(va[0][kb], va[1][kb], 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
      for (int tp = 0; tp < 9; ++tp)
        bfr[tp] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(vb[0][tp], vb[1][tp], 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int tp = 0; tp < 9; ++tp)
          acc[kb][tp] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[kb], bfr[tp], acc[kb][tp], 0, 0, 0);
    }
    if (tn >= ntile) break;
    t = tn;
  }
  dma_wait<0>();
  // partial slab: ws[blockIdx][k][tap*64 + c]
  float* out = a.ws + (size_t)blockIdx.x * C * 9 * C;
#pragma unroll
  for (int kb = 0; kb < 4; ++kb)
#pragma unroll
    for (int tp = 0; tp < 9; ++tp)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = kb * 16 + (lane >> 4) * 4 + r;
        out[(size_t)k * (9 * C) + tp * C + wid * 16 + (lane & 15)] = acc[kb][tp][r];
      }
}

}  // namespace dbx

using namespace dbx;

// Geometry the patch kernel covers: 3x3, stride 1, pad 1, 64 -> 64 channels, width 56, H % 8 == 0.
extern "C" int dbx_conv_patch3(int mode, const IGemmArgs* args, int pro, int stats, int epi, hipStream_t st,
                               int streamed) {
  const IGemmArgs& a = *args;
  if (a.R != 3 || a.S != 3 || a.stride != 1 || a.pad != 1 || a.IC != 64 || a.OC != 64) return -20;
  if (a.OW != 56 || a.IW != 56 || a.OH != a.IH || a.OH % 8 != 0) return -21;
  if (streamed) {  // patch3s_kernel: 4-row tiles, one per workgroup, two workgroups per CU
    const dim3 g(a.N * a.OH / 4), b(256);
    if (mode == FWD) {
      if (epi) return -22;
      if (pro && stats) hipLaunchKernelGGL((patch3s_kernel<FWD, true, true, 0, 4, 56>), g, b, 0, st, a);
      else if (pro) hipLaunchKernelGGL((patch3s_kernel<FWD, true, false, 0, 4, 56>), g, b, 0, st, a);
      else if (stats) hipLaunchKernelGGL((patch3s_kernel<FWD, false, true, 0, 4, 56>), g, b, 0, st, a);
      else hipLaunchKernelGGL((patch3s_kernel<FWD, false, false, 0, 4, 56>), g, b, 0, st, a);
    } else if (mode == DGRAD) {
      if (pro || stats || epi == 1 || a.osub != 1 || a.addsrc) return -22;
      if (epi == 2) hipLaunchKernelGGL((patch3s_kernel<DGRAD, false, false, 2, 4, 56>), g, b, 0, st, a);
      else hipLaunchKernelGGL((patch3s_kernel<DGRAD, false, false, 0, 4, 56>), g, b, 0, st, a);
    } else {
      return -24;
    }
    return (int)hipGetLastError();
  }
  const int ntile = a.N * a.OH / 8;
  static const int cus = [] {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return n > 0 ? n : 256;
  }();
  const int nwg = ntile < cus ? ntile : cus;
  if (mode == FWD) {
    if (epi) return -22;
    if (pro && stats) hipLaunchKernelGGL((patch3_kernel<FWD, true, true, 0, 8, 56>), dim3(nwg), dim3(512), 0, st, a);
    else if (pro) hipLaunchKernelGGL((patch3_kernel<FWD, true, false, 0, 8, 56>), dim3(nwg), dim3(512), 0, st, a);
    else if (stats) hipLaunchKernelGGL((patch3_kernel<FWD, false, true, 0, 8, 56>), dim3(nwg), dim3(512), 0, st, a);
    else hipLaunchKernelGGL((patch3_kernel<FWD, false, false, 0, 8, 56>), dim3(nwg), dim3(512), 0, st, a);
  } else if (mode == DGRAD) {
    if (pro || stats || epi == 1) return -22;
    if (a.osub != 1 || a.addsrc) return -23;
    if (epi == 2) hipLaunchKernelGGL((patch3_kernel<DGRAD, false, false, 2, 8, 56>), dim3(nwg), dim3(512), 0, st, a);
    else hipLaunchKernelGGL((patch3_kernel<DGRAD, false, false, 0, 8, 56>), dim3(nwg), dim3(512), 0, st, a);
  } else {
    return -24;
  }
  return (int)hipGetLastError();
}

// Stem (7x7 s2 p3, NHWC4 image of width 224 -> 64 channels at 112x112): the patch kernel above.
extern "C" int dbx_stem_patch(const IGemmArgs* args, int stats, hipStream_t st) {
  const IGemmArgs& a = *args;
  if (a.R != 7 || a.S != 7 || a.stride != 2 || a.pad != 3 || a.IC != 4 || a.OC != 64) return -30;
  if (a.IW != 224 || a.OW != 112 || a.OH % 4 != 0 || a.OH != (a.IH + 6 - 7) / 2 + 1) return -31;
  const int ntile = a.N * a.OH / 4;
  static const int cus = [] {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return n > 0 ? n : 256;
  }();
  const int nwg = ntile < cus ? ntile : cus;
  if (stats) hipLaunchKernelGGL((stem_patch_kernel<true, 4>), dim3(nwg), dim3(512), 0, st, a);
  else hipLaunchKernelGGL((stem_patch_kernel<false, 4>), dim3(nwg), dim3(512), 0, st, a);
  return (int)hipGetLastError();
}

// Weight gradient of the 64 -> 64 3x3 stride-1 convs at width 56: the patch kernel above writes
// one fp32 slab per workgroup into ws; returns the slab count (the caller reduces), < 0 on error.
// max_wg > 0: at most that many persistent workgroups (a side-stream launch leaving CUs free)
extern "C" int dbx_wgrad_patch3(const WgradArgs* args, long long ws_cap, hipStream_t st, int max_wg) {
  const WgradArgs& a = *args;
  if (a.R != 3 || a.S != 3 || a.stride != 1 || a.pad != 1 || a.IC != 64 || a.OC != 64) return -40;
  if (a.OW != 56 || a.IW != 56 || a.OH != a.IH || a.OH % 4 != 0) return -41;
  const int ntile = a.N * a.OH / 4;
  static const int cus = [] {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return n > 0 ? n : 256;
  }();
  const int cap = (max_wg > 0 && max_wg < cus) ? max_wg : cus;
  const int nwg = ntile < cap ? ntile : cap;
  // one slab per workgroup + the caller's two-level reduction partials (<= 64 slabs)
  if ((long long)(nwg + (nwg < 64 ? nwg : 64)) * a.OC * a.R * a.S * a.IC > ws_cap) return -42;
  hipLaunchKernelGGL((wgrad_patch3_kernel<4, 56>), dim3(nwg), dim3(256), 0, st, a);
  const int e = (int)hipGetLastError();
  return e ? -e : nwg;
}
