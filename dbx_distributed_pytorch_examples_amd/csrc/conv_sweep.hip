// N-sweep 1x1 forward with a BN prologue (tile code dma 8): the bottleneck conv3 expansions
// C -> 4C, Y = conv1x1(relu(X*scale + shift)) + this layer's BN statistics.
//
// The implicit-GEMM kernel (conv_igemm_kernel.h) walks 128 x 256 output tiles; the N / 256 tiles of
// one 128-row block each re-load the block's A operand (all K input channels), re-apply the BN
// prologue to it and re-stage it through LDS. At K = 128-256 that re-staging is most of the K loop
// (tools/probe_sweep.py: 1.3-1.7 us per 64-channel block and tile against 0.43 us of MFMA work), and
// the tile's epilogue is what remains. Here one workgroup owns a 128-row block for ALL output
// channels: the block's A operand is loaded from HBM once, transformed once and kept resident in LDS
// (128 x K bf16, <= 64 KiB at K = 256), and the workgroup sweeps the N / 256 sub-tiles over it --
// each sub-tile's K loop streams only the weights (L2-resident, [OC][K] <= 512 KiB) through a 2-slot
// LDS-DMA ring. Tensors stay resident instead of being re-read (cdna_hip_programming.md rule "keep
// tensors resident"); the MFMA schedule and the epilogue are those of the 128 x 256 igemm tile
// (igemm_epilogue, 2 x 4 waves of 64 x 64), so outputs and BN statistics are bit-identical to it.
//
// LDS: [KB][128][64] resident A | a region shared by the weight ring [2][256][64] and the epilogue's
// C staging [128][264] | the prologue affine [2][256] fp32  -> 132 KiB at K = 256: one workgroup per
// CU (8 waves), persistent over the 128-row blocks (grid = CUs, a multiple of 8: block b on XCD b % 8).
// The next block's A loads are issued during the last sub-tile's K loop (after its last weight DMA,
// so the counted ring waits never wait on them) and land while that sub-tile's epilogue runs.
#include "conv_igemm_kernel.h"

namespace dbx {

template <int KB, bool STATS>
__global__ __launch_bounds__(512, 1) void sweep_fwd_kernel(const IGemmArgs a) {
  constexpr int BM = 128, BN = 256, WM = 2, WN = 4, NT = 512, NW = 8, BK = 64;
  constexpr int CPR = BK / 8;               // 16-B chunks per 64-channel row
  constexpr int RPP = NT / CPR;             // rows per staging pass (64)
  constexpr int A_CH = BM * BK / 8 / NT;    // A chunks per thread and K block (2)
  constexpr int B_CH = BN * BK / 8 / NT;    // weight DMA instructions per wave and K block (4)
  constexpr int TM = BM / (16 * WM), TN = BN / (16 * WN);  // 4 x 4 MFMA tiles per wave
  constexpr int KMAX = KB * BK;
  constexpr int LDS_A = KB * BM * BK;                       // bf16 elements
  constexpr int LDS_RING = 2 * BN * BK;
  constexpr int LDS_C = BM * (BN + 8);
  constexpr int LDS_R = LDS_RING > LDS_C ? LDS_RING : LDS_C;
  __shared__ __attribute__((aligned(1024))) bf16 lds[LDS_A + LDS_R + 2 * 2 * KMAX];
  bf16* sA = lds;
  bf16* sR = lds + LDS_A;                                    // weight ring / C staging
  float* sPro = reinterpret_cast<float*>(lds + LDS_A + LDS_R);  // [2][KMAX] scale, shift

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wm = wid / WN, wn = wid % WN;
  const int ntm = (a.M + BM - 1) / BM, NJ = a.OC / BN;
  const int ach = tid & (CPR - 1);
  const int lch = ach ^ fswz<BK>(tid / CPR);  // weight DMA: the source chunk of this lane's LDS slot

  for (int c = tid; c < KMAX; c += NT) {
    sPro[c] = a.in_scale[c];
    sPro[KMAX + c] = a.in_shift[c];
  }
  const rsrc_t xr = make_rsrc(a.x, 2ull * a.M * a.IC);
  const i32x4 wsrd = make_srd(a.w, 2ull * a.OC * a.IC);
  const unsigned ring0 = lds_addr(sR);
  const u32x4 zero4 = {0u, 0u, 0u, 0u};

  u32x4 ra[KB][A_CH];
  auto load_a = [&](int t) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int m = t * BM + tid / CPR + RPP * i;
      const unsigned off = m < a.M ? 2u * (unsigned)(m * a.IC + ach * 8) : kOOB;  // rows past M: zeros
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) ra[kb][i] = buf_load16(xr, off == kOOB ? kOOB : off + 2u * kb * BK);
    }
  };
  // BN-apply + ReLU of the staged rows into the resident A image (padding rows stay exactly zero)
  auto stage_a = [&](int t) __attribute__((always_inline)) {
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      const int c0 = kb * BK + ach * 8;
      const f32x4 s0 = *reinterpret_cast<const f32x4*>(sPro + c0);
      const f32x4 s1 = *reinterpret_cast<const f32x4*>(sPro + c0 + 4);
      const f32x4 h0 = *reinterpret_cast<const f32x4*>(sPro + KMAX + c0);
      const f32x4 h1 = *reinterpret_cast<const f32x4*>(sPro + KMAX + c0 + 4);
#pragma unroll
      for (int i = 0; i < A_CH; ++i) {
        const int row = tid / CPR + RPP * i;
        float f[8];
        unpack8(ra[kb][i], f);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          f[j] = f[j] * s0[j] + h0[j];
          f[j + 4] = f[j + 4] * s1[j] + h1[j];
        }
        const u32x4 v = t * BM + row < a.M ? relu_bf16x8(pack8(f)) : zero4;
        *reinterpret_cast<u32x4*>(sA + kb * BM * BK + row * BK + ((ach ^ fswz<BK>(row)) << 3)) = v;
      }
    }
  };
  // weights of sub-tile j, K block kb -> ring slot s (LDS-DMA; the XOR swizzle on the source side)
  auto dma_b = [&](int j, int kb, int s) __attribute__((always_inline)) {
    const unsigned dst = ring0 + 2u * (unsigned)(s * BN * BK) + 1024u * (unsigned)wid;
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int n = j * BN + tid / CPR + RPP * i;
      lds_dma16(wsrd, 2u * (unsigned)(n * a.IC + kb * BK + lch * 8), dst + 1024u * (unsigned)(NW * i));
    }
  };

  f32x4 acc[TM][TN];
  auto mma = [&](int kb, int s) __attribute__((always_inline)) {
    const bf16* cA = sA + kb * BM * BK;
    const bf16* cB = sR + s * BN * BK;
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
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    }
  };

  int t = blockIdx.x;  // 128-row block (grid <= ntm: every workgroup has one)
  load_a(t);
  __syncthreads();  // sPro visible
  for (;;) {
    stage_a(t);      // (the previous block's last MFMA finished before its epilogue's first barrier)
    dma_b(0, 0, 0);  // the ring is free: the previous epilogue ended with a barrier
    const int tn = t + gridDim.x;
    for (int j = 0; j < NJ; ++j) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int jj = 0; jj < TN; ++jj) acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
        dma_wait<0>();     // this wave's part of block kb has landed (and everything older)
        __syncthreads();   // ... every wave's; slot (kb+1)&1 is no longer read; (kb 0: A image visible)
        if (kb + 1 < KB) dma_b(j, kb + 1, (kb + 1) & 1);
        else if (j + 1 == NJ && tn < ntm) load_a(tn);  // next block's A: lands under this epilogue
        mma(kb, kb & 1);
      }
      __syncthreads();  // every wave's MFMAs have read the ring before the epilogue stages C over it
      igemm_epilogue<BM, BN, WM, WN, FWD, STATS, false, 0>(a, acc, sR, t * BM, j * BN, t, blockIdx.x);
      // (ends with a barrier when STATS; a plain epilogue's last LDS reads precede its stores)
      if (!STATS) __syncthreads();
      if (j + 1 < NJ) dma_b(j + 1, 0, 0);
    }
    t = tn;
    if (t >= ntm) break;  // workgroup-uniform
  }
}

}  // namespace dbx

using namespace dbx;

// dma tile code 8 (ops/kernels.py conv_fwd): 1x1 stride-1 forward with a BN + ReLU prologue, K <= 256,
// OC % 256 == 0. Returns 0 or a negative code for an unsupported call (the host checks first).
extern "C" int dbx_conv_sweep(int mode, const IGemmArgs* args, int pro, int stats, int accum, int epi,
                              hipStream_t st) {
  const IGemmArgs& a = *args;
  if (mode != FWD || !pro || accum || epi || a.res || a.fin_in || a.ksplit > 1) return -70;
  if (a.R != 1 || a.S != 1 || a.stride != 1 || a.pad != 0 || !a.relu_in) return -71;
  if (a.IC % 64 != 0 || a.IC > 256 || a.OC % 256 != 0 || a.M <= 0) return -72;
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  const int ntm = (a.M + 127) / 128;
  const int grid = ntm < cus ? ntm : (cus & ~7);
#define SWEEP(KB_)                                                                                  \
  if (a.IC == 64 * KB_) {                                                                           \
    if (stats) hipLaunchKernelGGL((sweep_fwd_kernel<KB_, true>), dim3(grid), dim3(512), 0, st, a);  \
    else hipLaunchKernelGGL((sweep_fwd_kernel<KB_, false>), dim3(grid), dim3(512), 0, st, a);       \
    return (int)hipGetLastError();                                                                  \
  }
  SWEEP(1) SWEEP(2) SWEEP(3) SWEEP(4)
#undef SWEEP
  return -72;
}
