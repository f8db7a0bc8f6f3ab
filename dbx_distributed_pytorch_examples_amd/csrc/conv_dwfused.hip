// Fused backward of a bottleneck conv3 (1x1 stride 1, C -> K channels) in ONE pass over its
// output gradient (SURVEY.md §2.4 K4 + K5 + K7 for the bottleneck tail; the reference runs these
// as cuDNN dgrad, cuDNN wgrad and BatchNorm-backward kernels, each re-reading HBM).
//
// Per tile of BM output pixels, with a2 = relu(y2 * bsc + bsh) (the BN2 output = conv3's input):
//   dy3 = k1*g + k2*y3 + k3                 BN3-backward apply (per channel k), rounded to bf16
//   da  = [a2 > 0] * (dy3 . W)              data gradient -> out (bf16)
//   BN2 backward moments sum da, sum da*y2  (per workgroup in registers, fp64 atomics at the end)
//   dW += dy3^T . a2                        weight gradient (fp32, in registers across all tiles)
// dy3 and a2 only ever exist in LDS: compared with the unfused schedule (BN3 apply folded into the
// dgrad, which stores dy3 and a2, then a separate weight-gradient pass reading both) this removes
// writing and re-reading dy3 (2 x K channels per pixel) and a2 (2 x C), i.e. 10 of the 20 bytes
// per pixel-channel-unit the two kernels moved at the 56x56 stage (C = 64, K = 256).
//
// Workgroup = 4 waves (2 per CU x 2 workgroups), persistent over tiles t = blockIdx.x + i*grid.
// LDS: the whole dgrad weight [C][K] resident (loaded once), dy3 K-blocks double-buffered, the a2
// tile. dy3 / a2 images use the wgrad tr_swz swizzle, which is conflict-free for the ds_write_b128
// staging, the dgrad fragments (ds_read_b128 along k) and the wgrad fragments (ds_read_b64_tr_b16
// along pixels) alike (exhaustive check: tools/lds_banks.py). Each workgroup writes one fp32
// partial slab of dW; wgrad_reduce sums them in a fixed order (deterministic).
#include "common.h"
#include "abi.h"

namespace dbx {

// C: dgrad output channels (conv3 input), NKB: K / 64, BM: pixels per tile, NS: register staging
// sets (the g / y3 loads of block kb + NS are issued while block kb is computed), NT: threads,
// WN: waves along the channels (grid 2 x WN: a wave owns C / WN channels of both GEMMs, so the
// weight-gradient accumulators per lane are 64 K / NT x C), OCC: workgroups per CU, Y2N: prefetch the
// next tile's y2 into spare registers at the tile start (else during the epilogue).
template <int C, int NKB, int BM, int NS, int NT, int WN, int OCC, bool Y2N>
__global__ __launch_bounds__(NT, OCC) void dwfused_kernel(const DwFusedArgs a) {
  constexpr int K = NKB * 64;
  constexpr int NW = NT / 64, WM = NW / WN;  // wave grid: WM x WN (WM = 2)
  constexpr int WC = C / WN;                 // channels per wave
  constexpr int WCH = K / 8;            // 16-byte chunks per resident weight row
  constexpr int CPR = C / 8;            // chunks per a2 / da row
  constexpr int RPP = NT / CPR;         // a2 / da rows per thread pass
  constexpr int NY = BM / RPP;          // y2 / da chunks per thread
  constexpr int LR = NT / 8;            // g / y3 rows per thread pass (8 chunks per 64-wide row)
  constexpr int NG = BM / LR;           // g / y3 chunks per thread and K-block (rows lrow + LR i)
  constexpr int TM = BM / (16 * WM), TN = WC / 16;  // dgrad: wave (wm, wn) owns BM/WM pixels x WC channels
  constexpr int TNW = WC / 16;                      // wgrad: wave owns 32 k x WC channels of each K-block
  static_assert(NKB % NS == 0 && C % 64 == 0 && WM == 2 && BM % (16 * WM) == 0 && BM % LR == 0 && BM % RPP == 0,
                "tile shape");
  constexpr int LDS_W = C * K, LDS_A = 2 * BM * 64, LDS_P = BM * C;
  static_assert(BM * (C + 8) <= LDS_A + LDS_P, "epilogue staging must fit the dy3 + a2 images");
  __shared__ __attribute__((aligned(16))) bf16 lds[LDS_W + LDS_A + LDS_P];
  bf16* sW = lds;              // [C][K], chunk ^ (row & 15)
  bf16* sA = lds + LDS_W;      // [2][BM][64] dy3 K-blocks (tr_swz)
  bf16* sP = sA + LDS_A;       // [BM][C] a2 tile (tr_swz)
  bf16* sC = sA;               // epilogue staging [BM][C + 8] (aliases sA + sP after the K loop)

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wm = wid / WN, wn = wid % WN;
  const int ntile = a.M / BM;
  const int lrow = tid >> 3, lch = tid & 7;      // g / y3 loader: rows lrow + LR i, chunk lch
  const int erow = tid / CPR, ech = tid % CPR;   // y2 / epilogue: rows erow + RPP i, chunk ech

  for (int q = tid; q < C * WCH; q += NT) {
    const int row = q / WCH, ch = q - (q / WCH) * WCH;
    *reinterpret_cast<u32x4*>(sW + row * K + ((ch ^ (row & 15)) << 3)) =
        *reinterpret_cast<const u32x4*>(a.wt + (size_t)row * K + ch * 8);
  }
  // BN2 forward affine of this thread's 8 channels: re-read (L1 / L2 hits) at each use instead of
  // pinning 16 VGPRs across the K loop (the accumulators need them)
  int cbn = ech * 8;
  auto bn2_affine = [&](f32x4& s0, f32x4& s1, f32x4& h0, f32x4& h1) __attribute__((always_inline)) {
    asm volatile("" : "+v"(cbn));  // opaque: keeps the loads at the use (not hoisted out of the tile loop)
    s0 = *reinterpret_cast<const f32x4*>(a.bsc + cbn);
    s1 = *reinterpret_cast<const f32x4*>(a.bsc + cbn + 4);
    h0 = *reinterpret_cast<const f32x4*>(a.bsh + cbn);
    h1 = *reinterpret_cast<const f32x4*>(a.bsh + cbn + 4);
  };
  f32x2 st_s[4], st_q[4];  // running BN2-backward raw moments of this thread's channels (packed)
#pragma unroll
  for (int h = 0; h < 4; ++h) st_s[h] = st_q[h] = f32x2{0.f, 0.f};
  f32x4 accw[NKB][2][TNW];
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < TNW; ++j) accw[kb][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const rsrc_t gr = make_rsrc(a.g, 2ull * a.M * K);
  const rsrc_t yr = make_rsrc(a.y3, 2ull * a.M * K);
  const rsrc_t y2r = make_rsrc(a.y2, 2ull * a.M * C);
  u32x4 rg[NS][NG], ry[NS][NG], ry2[NY], ry2n[Y2N ? NY : 1];
  // tiles past the end read out of range (zeros, no traffic): the prefetch is unconditional
  auto load_k = [&](int t, int kb, int set) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NG; ++i) {
      const unsigned off = t < ntile ? 2u * (unsigned)((t * BM + lrow + LR * i) * K + kb * 64 + lch * 8) : kOOB;
      rg[set][i] = buf_load16(gr, off);
      ry[set][i] = buf_load16(yr, off);
    }
  };
  auto y2_off = [&](int t, int i) __attribute__((always_inline)) {
    return t < ntile ? 2u * (unsigned)((t * BM + erow + RPP * i) * C + ech * 8) : kOOB;
  };
  // BN3-backward apply of K-block kb -> dy3 image (bf16, as the unfused fold stores it)
  auto fold_store = [&](int kb, int buf, int set) __attribute__((always_inline)) {
    const int c0 = kb * 64 + lch * 8;
    const f32x4 k1a = *reinterpret_cast<const f32x4*>(a.coeff + c0);
    const f32x4 k1b = *reinterpret_cast<const f32x4*>(a.coeff + c0 + 4);
    const f32x4 k2a = *reinterpret_cast<const f32x4*>(a.coeff + K + c0);
    const f32x4 k2b = *reinterpret_cast<const f32x4*>(a.coeff + K + c0 + 4);
    const f32x4 k3a = *reinterpret_cast<const f32x4*>(a.coeff + 2 * K + c0);
    const f32x4 k3b = *reinterpret_cast<const f32x4*>(a.coeff + 2 * K + c0 + 4);
#pragma unroll
    for (int i = 0; i < NG; ++i) {
      float f[8], y[8];
      unpack8(rg[set][i], f);
      unpack8(ry[set][i], y);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        f[j] = f[j] * k1a[j] + k3a[j] + y[j] * k2a[j];
        f[j + 4] = f[j + 4] * k1b[j] + k3b[j] + y[j + 4] * k2b[j];
      }
      const int row = lrow + LR * i;
      *reinterpret_cast<u32x4*>(sA + buf * BM * 64 + row * 64 + (tr_swz(row, lch, 8) << 3)) = pack8(f);
    }
  };
  auto a2_store = [&]() __attribute__((always_inline)) {
    f32x4 bsc0, bsc1, bsh0, bsh1;
    bn2_affine(bsc0, bsc1, bsh0, bsh1);
#pragma unroll
    for (int i = 0; i < NY; ++i) {
      float f[8];
      unpack8(ry2[i], f);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        f[j] = f[j] * bsc0[j] + bsh0[j];
        f[j + 4] = f[j + 4] * bsc1[j] + bsh1[j];
      }
      const int row = erow + RPP * i;
      *reinterpret_cast<u32x4*>(sP + row * C + (tr_swz(row, ech, CPR) << 3)) = relu_bf16x8(pack8(f));
    }
  };

  const int g4 = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
  f32x4 accd[TM][TN];
  auto mma = [&](int kb, int buf) __attribute__((always_inline)) {
    const bf16* cA = sA + buf * BM * 64;
    // data gradient: acc^T = W . dy3^T (a lane's 4 accumulators = 4 consecutive channels of a pixel)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ch = ks * 4 + g4;
      bf16x8 af[TM], bw[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * (BM / WM) + i * 16 + (lane & 15);
        af[i] = *reinterpret_cast<const bf16x8*>(cA + row * 64 + (tr_swz(row, ch, 8) << 3));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int crow = wn * WC + j * 16 + (lane & 15);
        bw[j] = *reinterpret_cast<const bf16x8*>(sW + crow * K + (((kb * 8 + ch) ^ (crow & 15)) << 3));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          accd[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[j], af[i], accd[i][j], 0, 0, 0);
    }
    // weight gradient of this K-block: dW[k][c] += sum_m dy3[m][k] * a2[m][c]  (reduction over
    // the tile's pixels in steps of 32; fragments by hardware-transposed LDS reads)
#pragma unroll
    for (int ks = 0; ks < BM / 32; ++ks) {
      const int row = ks * 32 + 8 * g4 + q4, row2 = row + 4;
      bf16x8 af[2], bp[TNW];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int col = wm * 32 + i * 16 + 4 * p4;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (DBX_LDS s16x4*)(cA + row * 64 + (tr_swz(row, col >> 3, 8) << 3) + (col & 7)));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (DBX_LDS s16x4*)(cA + row2 * 64 + (tr_swz(row2, col >> 3, 8) << 3) + (col & 7)));
        af[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int j = 0; j < TNW; ++j) {
        const int col = wn * WC + j * 16 + 4 * p4;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (DBX_LDS s16x4*)(sP + row * C + (tr_swz(row, col >> 3, CPR) << 3) + (col & 7)));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (DBX_LDS s16x4*)(sP + row2 * C + (tr_swz(row2, col >> 3, CPR) << 3) + (col & 7)));
        bp[j] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < TNW; ++j)
          accw[kb][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bp[j], accw[kb][i][j], 0, 0, 0);
    }
  };

  int t = blockIdx.x;
#pragma unroll
  for (int i = 0; i < NY; ++i) ry2[i] = buf_load16(y2r, y2_off(t, i));
#pragma unroll
  for (int s = 0; s < NS; ++s) load_k(t, s, s);
  __syncthreads();  // resident weights visible
  for (; t < ntile; t += gridDim.x) {
    const int tn = t + gridDim.x;
    if constexpr (Y2N) {
#pragma unroll
      for (int i = 0; i < NY; ++i) ry2n[i] = buf_load16(y2r, y2_off(tn, i));
    }
    a2_store();
    fold_store(0, 0, 0);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) accd[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb) {
      // register set kb % NS was consumed by fold_store(kb): refill it with the block NS ahead in
      // the stream (past the tile's last block: the next tile's first blocks), under kb's MFMAs
      const int f = kb + NS;
      load_k(f < NKB ? t : tn, f < NKB ? f : f - NKB, kb % NS);
      mma(kb, kb & 1);
      if (kb + 1 < NKB) fold_store(kb + 1, (kb + 1) & 1, (kb + 1) % NS);
      __syncthreads();
    }
    // epilogue: da = [a2 > 0] * acc, staged through LDS for 16-byte row chunks (the thread's chunks
    // are the rows / channels of its y2 registers)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wm * (BM / WM) + i * 16 + (lane & 15);
        const int col = wn * WC + j * 16 + g4 * 4;
        *reinterpret_cast<uint2*>(sC + row * (C + 8) + col) =
            uint2{pack2(accd[i][j][0], accd[i][j][1]), pack2(accd[i][j][2], accd[i][j][3])};
      }
    __syncthreads();
    f32x4 bsc0, bsc1, bsh0, bsh1;
    bn2_affine(bsc0, bsc1, bsh0, bsh1);
#pragma unroll
    for (int i = 0; i < NY; ++i) {
      const int row = erow + RPP * i;
      float f[8], y[8];
      unpack8(*reinterpret_cast<const u32x4*>(sC + row * (C + 8) + ech * 8), f);
      unpack8(ry2[i], y);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float t0 = y[j] * bsc0[j] + bsh0[j], t1 = y[j + 4] * bsc1[j] + bsh1[j];
        f[j] = t0 > 0.f ? f[j] : 0.f;
        f[j + 4] = t1 > 0.f ? f[j + 4] : 0.f;
      }
      const u32x4 v = pack8(f);
      *reinterpret_cast<u32x4*>(a.da + (size_t)(t * BM + row) * C + ech * 8) = v;
#pragma unroll
      for (int h = 0; h < 4; ++h) {  // raw moments of the stored (bf16) values: sum g, sum g*y2
        const f32x2 gv = {__uint_as_float(v[h] << 16), __uint_as_float(v[h] & 0xFFFF0000u)};
        const f32x2 yv = {__uint_as_float(ry2[i][h] << 16), __uint_as_float(ry2[i][h] & 0xFFFF0000u)};
        st_s[h] += gv;
        st_q[h] = __builtin_elementwise_fma(gv, yv, st_q[h]);
      }
      // the next tile's y2: prefetched at the tile start (Y2N) or now, into the register just consumed
      if constexpr (Y2N) ry2[i] = ry2n[i];
      else ry2[i] = buf_load16(y2r, y2_off(tn, i));
    }
    __syncthreads();  // sC (= sA + sP) free for the next tile's staging
  }

  // weight-gradient partial slab ws[blockIdx][k][c] (every workgroup writes one, zero if it had no tile)
  float* out = a.ws + (size_t)blockIdx.x * K * C;
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < TNW; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int k = kb * 64 + wm * 32 + i * 16 + g4 * 4 + r;
          out[(size_t)k * C + wn * WC + j * 16 + (lane & 15)] = accw[kb][i][j][r];
        }
  // BN2-backward moments: threads with the same chunk column (lanes l, l ^ CPR, ...; then the 4 waves
  // through LDS), centred once per channel: sum g*xhat = inv * (sum g*y - mean * sum g)
  float s[8], q[8];
#pragma unroll
  for (int h = 0; h < 4; ++h) {
    s[2 * h] = st_s[h].x; s[2 * h + 1] = st_s[h].y;
    q[2 * h] = st_q[h].x; q[2 * h + 1] = st_q[h].y;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int o = CPR; o < 64; o <<= 1) {
      s[j] += __shfl_xor(s[j], o, 64);
      q[j] += __shfl_xor(q[j], o, 64);
    }
  float* red = reinterpret_cast<float*>(sA);  // [NW waves][2][C] (the loop's last barrier freed sA)
  if (lane < CPR) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[(wid * 2 + 0) * C + lane * 8 + j] = s[j];
      red[(wid * 2 + 1) * C + lane * 8 + j] = q[j];
    }
  }
  __syncthreads();
  for (int c = tid; c < C; c += NT) {
    float ss = 0.f, qq = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) { ss += red[(w * 2) * C + c]; qq += red[(w * 2 + 1) * C + c]; }
    qq = a.inv2[c] * (qq - a.mean2[c] * ss);
    double* st = a.bstats + (size_t)(blockIdx.x % a.nshard) * 2 * C;
    atomicAdd(st + c, (double)ss);
    atomicAdd(st + C + c, (double)qq);
  }
}

}  // namespace dbx

using namespace dbx;

// Returns the number of partial slabs written (= workgroups), or a negative error.
template <int C, int NKB, int BM, int NS, int NT, int WN, int OCC, bool Y2N>
static int launch_dwfused(const DwFusedArgs& a, long long ws_cap, hipStream_t st, int max_cus) {
  if (a.M % BM != 0 || a.M <= 0) return -31;
  struct Occ { int per_cu, cus; };
  static const Occ occ = [] {
    int per_cu = 0, dev = 0, cus = 0;
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &per_cu, reinterpret_cast<const void*>(&dwfused_kernel<C, NKB, BM, NS, NT, WN, OCC, Y2N>), NT, 0);
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    return Occ{per_cu, cus};
  }();
  // max_cus > 0: the persistent grid spans only that many CUs (a multiple of 8: XCD round-robin), the
  // rest stay with a concurrent side stream
  const int cus = (max_cus > 0 && max_cus < occ.cus) ? (max_cus & ~7) : occ.cus;
  const int cap = (occ.per_cu > 0 && cus > 0) ? occ.per_cu * cus : 256;
  const int ntile = a.M / BM;
  const int grid = ntile < cap ? ntile : cap;
  if ((long long)(grid + (grid < 64 ? grid : 64)) * a.K * a.C > ws_cap) return -33;
  hipLaunchKernelGGL((dwfused_kernel<C, NKB, BM, NS, NT, WN, OCC, Y2N>), dim3(grid), dim3(NT), 0, st, a);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? grid : -(int)e - 1000;
}

// ws_cap: floats available at a.ws (the slabs plus wgrad_reduce's level-1 partials); max_cus: see
// launch_dwfused (0: all CUs).
// Returns the number of partial slabs written (= workgroups), or a negative error.
extern "C" int dbx_conv_dwfused(const DwFusedArgs* args, long long ws_cap, hipStream_t st, int max_cus) {
  const DwFusedArgs& a = *args;
  if (2ull * a.M * a.K >= (unsigned long long)kOOB) return -32;  // 32-bit buffer offsets
  // 56x56 stage: two workgroups per CU (32 KB resident weights), 64-pixel tiles, two register sets
  // (0.903 ms at b1024 vs 0.928 ms for 128-pixel tiles with one set, 1.052 ms with 64 / one set)
#ifndef DBX_DWF64
#define DBX_DWF64 64, 2, 256, 2, 2, false
#endif
  if (a.C == 64 && a.K == 256) return launch_dwfused<64, 4, DBX_DWF64>(a, ws_cap, st, max_cus);
  // 28x28 stage: 128 KB resident weights -> one workgroup per CU; 4 waves (2 x 2) whose lanes hold
  // the 256 weight-gradient accumulators in AGPRs, 64-pixel tiles, two register sets in flight.
  // Measured at b1024 (tools/bench_dwfused.py, profiles/r2s4_dwfused/): 0.631 ms vs 0.875 ms with
  // 32-pixel tiles, 0.73 / 1.03 ms with 8 waves (2 x 4, 128 accumulators per lane, 2 / 4 sets: the
  // rest of the state still spills at 256 registers), 0.811 ms for the unfused dgrad + wgrad pair
#ifndef DBX_DWF128
#define DBX_DWF128 64, 2, 256, 2, 1, false
#endif
  if (a.C == 128 && a.K == 512) return launch_dwfused<128, 8, DBX_DWF128>(a, ws_cap, st, max_cus);
  return -30;
}
