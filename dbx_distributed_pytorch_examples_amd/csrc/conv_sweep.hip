// N-sweep 1x1 convs (tile code dma 8): the bottleneck conv3 expansions C -> 4C with their BN + ReLU
// prologue and BN statistics, and the conv1 data gradients 4C <- C with the
// BN1-backward apply folded into the operand and the previous block's BN-backward epilogue (K4, K7).
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
// The next block's A loads are issued at the last K step of the last sub-tile (after its last weight
// DMA: no ring wait of this block waits on them) and land while that sub-tile's epilogue runs.
// Measured and rejected variants: deferred epilogue stores (r6_defer/), a 4-slot ring of 32-channel
// weight stages (r6_ring4/).
#include "conv_igemm_kernel.h"

namespace dbx {

// MODE FWD: A = relu(x*scale + shift) (BN + ReLU prologue), STATS: this layer's BN statistics.
// MODE DGRAD (TAIL): the bottleneck conv1 data gradient with the BN1-backward apply folded in --
// A = g*k1 + k3 + y*k2 (x = g, res = y; no ReLU), stored once per row block to tail_out (the weight
// gradient's dy); ACCUM: + the block-input addend; EPI 1: the previous block's MASK_OUT epilogue (the
// data-gradient mode is 1.08-1.23x per launch but neutral inside the step: engine default off,
// profiles/r6_sweep/).
// APF: the next row block's A loads are issued under the last sub-tile (register room permitting).
template <int KB, int MODE, bool STATS, bool ACCUM, int EPI, bool TAIL>
__global__ __launch_bounds__(512, 1) void sweep_kernel(const IGemmArgs a) {
  constexpr int BM = 128, BN = 256, WM = 2, WN = 4, NT = 512, NW = 8, BK = 64;
  constexpr int CPR = BK / 8;               // 16-B chunks per 64-channel row
  constexpr int RPP = NT / CPR;             // rows per staging pass (64)
  constexpr int A_CH = BM * BK / 8 / NT;    // A chunks per thread and K block (2)
  constexpr int B_CH = BN * BK / 8 / NT;    // weight DMA instructions per wave and K block (4)
  constexpr int TM = BM / (16 * WM), TN = BN / (16 * WN);  // 4 x 4 MFMA tiles per wave
  constexpr int KMAX = KB * BK;
  constexpr int NPRO = TAIL ? 4 : 2;        // prologue affine arrays
  constexpr bool APF = !TAIL || KB == 1;  // (TAIL at KB >= 2: no register room beside the EPI epilogue)
  constexpr int LDS_A = KB * BM * BK;                       // bf16 elements
  constexpr int LDS_RING = 2 * BN * BK;
  constexpr int LDS_C = BM * (BN + 8);                      // (>= the EPI reduction scratch, which reuses it)
  constexpr int LDS_R = LDS_RING > LDS_C ? LDS_RING : LDS_C;
  static_assert(3 * NW * BN * 4 <= LDS_C * 2, "EPI reduction scratch inside the C staging");
  __shared__ __attribute__((aligned(1024))) bf16 lds[LDS_A + LDS_R + 2 * NPRO * KMAX];
  bf16* sA = lds;
  bf16* sR = lds + LDS_A;                                    // weight ring / C staging
  float* sPro = reinterpret_cast<float*>(lds + LDS_A + LDS_R);  // [NPRO][KMAX]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wm = wid / WN, wn = wid % WN;
  const int ntm = (a.M + BM - 1) / BM, NJ = a.OC / BN;
  const int ach = tid & (CPR - 1);
  const int lch = ach ^ fswz<BK>(tid / CPR);  // weight DMA: the source chunk of this lane's LDS slot

  for (int c = tid; c < KMAX; c += NT) {
    sPro[c] = a.in_scale[c];
    sPro[KMAX + c] = a.in_shift[c];
    if constexpr (TAIL) {
      sPro[2 * KMAX + c] = a.res_scale ? a.res_scale[c] : 1.f;
      sPro[3 * KMAX + c] = a.res_shift ? a.res_shift[c] : 0.f;
    }
  }
  const rsrc_t xr = make_rsrc(a.x, 2ull * a.M * a.IC);
  const rsrc_t rr_ = make_rsrc(a.res, TAIL ? 2ull * a.M * a.IC : 0ull);
  const rsrc_t toutr = make_rsrc(a.tail_out, (TAIL && a.tail_out) ? 2ull * a.M * a.IC : 0ull);
  const i32x4 wsrd = make_srd(a.w, 2ull * a.OC * a.IC);
  const unsigned ring0 = lds_addr(sR);
  const u32x4 zero4 = {0u, 0u, 0u, 0u};

  u32x4 ra[KB][A_CH], rr[TAIL ? KB : 1][A_CH];
  auto load_a = [&](int t) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int m = t * BM + tid / CPR + RPP * i;
      const unsigned off = m < a.M ? 2u * (unsigned)(m * a.IC + ach * 8) : kOOB;  // rows past M: zeros
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
        const unsigned o = off == kOOB ? kOOB : off + 2u * kb * BK;
        ra[kb][i] = buf_load16(xr, o);
        if constexpr (TAIL) rr[kb][i] = buf_load16(rr_, o);
      }
    }
  };
  // the prologue on the staged rows into the resident A image (padding rows stay exactly zero); TAIL
  // also stores the transformed rows (tail_out: the weight gradient's operand)
  auto stage_a = [&](int t) __attribute__((always_inline)) {
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      const int c0 = kb * BK + ach * 8;
#pragma unroll
      for (int i = 0; i < A_CH; ++i) {
        const int row = tid / CPR + RPP * i;
        const bool live = t * BM + row < a.M;
        float f[8];
        unpack8(ra[kb][i], f);
        if constexpr (TAIL) {
          float g[8];
          unpack8(rr[kb][i], g);
#pragma unroll
          for (int j = 0; j < 8; ++j)
            f[j] = f[j] * sPro[c0 + j] + sPro[KMAX + c0 + j] + (g[j] * sPro[2 * KMAX + c0 + j] + sPro[3 * KMAX + c0 + j]);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = f[j] * sPro[c0 + j] + sPro[KMAX + c0 + j];
        }
        u32x4 v = pack8(f);
        if constexpr (MODE != DGRAD) v = relu_bf16x8(v);
        v = live ? v : zero4;
        *reinterpret_cast<u32x4*>(sA + kb * BM * BK + row * BK + ((ach ^ fswz<BK>(row)) << 3)) = v;
        if constexpr (TAIL)
          buf_store16(toutr, live ? 2u * (unsigned)((t * BM + row) * a.IC + c0) : kOOB, v);
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
  if constexpr (APF) load_a(t);
  __syncthreads();  // sPro visible
  for (;;) {
    if constexpr (!APF) load_a(t);
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
        else if (APF && j + 1 == NJ && tn < ntm) load_a(tn);  // next block's A: lands under this epilogue
        mma(kb, kb & 1);
      }
      __syncthreads();  // every wave's MFMAs have read the ring before the epilogue stages C over it
      igemm_epilogue<BM, BN, WM, WN, MODE, STATS, ACCUM, EPI>(a, acc, sR, t * BM, j * BN, t, blockIdx.x);
      __syncthreads();  // the epilogue's last LDS reads before the ring is refilled
      if (j + 1 < NJ) dma_b(j + 1, 0, 0);
    }
    t = tn;
    if (t >= ntm) break;  // workgroup-uniform
  }
}

}  // namespace dbx

using namespace dbx;

// dma tile code 8 (ops/kernels.py conv_fwd / conv_dgrad): 1x1 stride-1 convs with K <= 256 staged input
// channels and OC % 256 == 0 -- the BN + ReLU prologue forward (+ statistics), or the folded
// BN-backward data gradient (TAIL: res = the BN input, tail_out = its stored output; + addend at full
// resolution; epilogue 0 / 1). Returns 0 or a negative code for an unsupported call.
template <int KB>
static int launch_sweep(int mode, const IGemmArgs& a, int stats, int accum, int epi, int grid, hipStream_t st) {
#define L(...) hipLaunchKernelGGL((sweep_kernel<KB, __VA_ARGS__>), dim3(grid), dim3(512), 0, st, a)
  if (mode == FWD) {
    if (stats) L(FWD, true, false, 0, false); else L(FWD, false, false, 0, false);
  } else if (accum) {
    if (epi == 1) L(DGRAD, false, true, 1, true); else L(DGRAD, false, true, 0, true);
  } else {
    if (epi == 1) L(DGRAD, false, false, 1, true); else L(DGRAD, false, false, 0, true);
  }
#undef L
  return (int)hipGetLastError();
}

extern "C" int dbx_conv_sweep(int mode, const IGemmArgs* args, int pro, int stats, int accum, int epi,
                              hipStream_t st) {
  const IGemmArgs& a = *args;
  if (!pro || a.fin_in || a.ksplit > 1 || a.R != 1 || a.S != 1 || a.stride != 1 || a.pad != 0) return -70;
  if (mode == FWD) {
    if (accum || epi || a.res || !a.relu_in) return -71;
  } else if (mode == DGRAD) {
    if (!a.res || stats || a.osub != 1 || (accum && a.add_sub != 1) || a.tail_bits) return -71;
    if (a.a_out || epi == 2) return -71;  // (the MASK_Y epilogue is not instantiated: no register room)
  } else {
    return -71;
  }
  if (a.IC % 64 != 0 || a.IC > 256 || a.OC % 256 != 0 || a.M <= 0) return -72;
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  // persistent grid: one workgroup per CU (LDS-bound occupancy), or a.kper when set (split-K is
  // never combined with this kernel, so the field carries the grid cap): > 0 caps the workgroups
  // (room for a concurrent side stream), < 0 launches one workgroup per row block (no persistence)
  const int ntm = (a.M + 127) / 128;
  int cap = a.kper > 0 ? a.kper : (cus & ~7);
  if (a.kper < 0) cap = ntm;
  const int grid = ntm < cap ? ntm : cap;
  switch (a.IC / 64) {
    case 1: return launch_sweep<1>(mode, a, stats, accum, epi, grid, st);
    case 2: return launch_sweep<2>(mode, a, stats, accum, epi, grid, st);
    case 3: return launch_sweep<3>(mode, a, stats, accum, epi, grid, st);
    case 4: return launch_sweep<4>(mode, a, stats, accum, epi, grid, st);
  }
  return -72;
}
