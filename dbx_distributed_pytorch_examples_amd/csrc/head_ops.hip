// Classifier-head kernels on CDNA4: the fc GEMMs (forward, data gradient, weight gradient) with
// fused bias / Philox dropout, the bias-gradient column sum, and the CutMix-aware soft-label
// pieces of the head (reference: `02_cifar_torch_distributor_resnet.py:153-156` Dropout(0.5) ->
// Linear head; torchvision fc).
//
// small_gemm: C[M][N] = alpha * sum_k A(m, k) * B(k, n) (+ bias[n]) (+ C)
//   A: TA = 0 -> [M][K] row-major (lda), TA = 1 -> [K][M] (lda)
//   B: TB = 0 -> [N][K] (ldb),          TB = 1 -> [K][N] (ldb)
// Tiles 64 x 64 x 128 per 4-wave workgroup (2 x 2 waves, 32 x 32 each = 2 x 2 v_mfma_f32_16x16x32_bf16),
// both operands staged into K-contiguous LDS images ([m][k], [n][k], XOR-swizzled 16-byte chunks) so
// every fragment is one ds_read_b128; transposed sources are transposed by the staging store.
// Shapes are arbitrary (masked edges): logits [B, 1000 | 200 | 10] = pooled [B, 2048 | 512] x W^T,
// dpooled = dlogits x W (reduction over the classes), dW = dlogits^T x h (reduction over the batch).
// These GEMMs are 0.1-0.3 % of a ResNet-50 step; the point is one native path with the dropout and
// bias fused, not peak MFMA rate. Long-K shapes with few tiles (the fc forward at batch 512 / 200
// classes: 32 tiles x 16 k-stages, 35 us on 32 of 256 CUs) split K over blockIdx.z into fp32 partials
// that split_gemm_reduce sums in split order and finishes (alpha, bias, accumulate, output type).
//
// Dropout (DROP = 1: on A, DROP = 2: on B): element at memory index i of that operand is kept with
// probability keep (scaled 1/keep) by a Philox-4x32-10 draw at counter (i / 4, seed_lo, seed_hi,
// offset): the backward regenerates exactly the forward's mask from (seed, offset), no mask tensor.
#include "common.h"
#include "abi.h"

namespace dbx {

// Philox-4x32-10 (Salmon et al., SC'11): counter-based, so any element's draw is recomputable.
__device__ __forceinline__ unsigned philox_u32(unsigned long long idx, unsigned long long seed, unsigned offset) {
  // counter (idx / 4 lo, idx / 4 hi, offset, 0), key = seed; element idx takes word idx % 4
  unsigned c0 = (unsigned)(idx >> 2), c1 = (unsigned)(idx >> 34), c2 = offset, c3 = 0u;
  unsigned k0 = (unsigned)seed, k1 = (unsigned)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const unsigned long long p0 = (unsigned long long)0xD2511F53u * c0;
    const unsigned long long p1 = (unsigned long long)0xCD9E8D57u * c2;
    const unsigned n0 = (unsigned)(p1 >> 32) ^ c1 ^ k0, n1 = (unsigned)p1;
    const unsigned n2 = (unsigned)(p0 >> 32) ^ c3 ^ k1, n3 = (unsigned)p0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  const unsigned w = (unsigned)(idx & 3);
  return w == 0 ? c0 : w == 1 ? c1 : w == 2 ? c2 : c3;
}

__device__ __forceinline__ float drop_scale(unsigned long long idx, unsigned long long seed, unsigned offset,
                                            unsigned thresh, float inv_keep) {
  return philox_u32(idx, seed, offset) < thresh ? inv_keep : 0.f;
}

template <int TA, int TB, bool OUT_F32, int DROP>
__global__ __launch_bounds__(256) void small_gemm_kernel(const GemmArgs g) {
  // 64 x 64 output tile, K staged 128 deep (4 MFMA k-steps per barrier pair) with the next stage's
  // global loads issued into registers before this stage's MFMAs: the head GEMMs have few tiles
  // (fc forward at batch 256 / 10 classes: 4 workgroups) and are latency-bound on the K loop, so
  // the loop is cut to K / 128 iterations, each hiding the next stage's load latency.
  constexpr int BM = 64, BN = 64, BK = 128, NCH = BK / 8, CPT = BM * NCH / 256;  // 4 chunks / thread
  __shared__ __attribute__((aligned(16))) bf16 sA[BM * BK];
  __shared__ __attribute__((aligned(16))) bf16 sB[BN * BK];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wm = wid >> 1, wn = wid & 1;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  // split-K: this workgroup's K range (multiples of BK; the last split takes the rest)
  const int kper = g.splitk > 1 ? ((g.K + g.splitk - 1) / g.splitk + BK - 1) / BK * BK : g.K;
  const int kbeg = (int)blockIdx.z * kper, kend = min(g.K, kbeg + kper);
  const unsigned doff = (DROP && g.offset_dev) ? *g.offset_dev : g.offset;  // step counter (device)
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // staging: chunk q = tid + 256 c (c < 4) -> (row = q / 16, chunk = q % 16) of the K-contiguous
  // image [64][128]; chunk ^ (row & 15) spreads 16 consecutive rows of one k chunk over all 64 banks
  auto swz = [](int row, int ch) { return ch ^ (row & 15); };
  // 8 elements (k = k0 + 8 ch .. +7) of operand row r0 + row (dropout applied, zeros past the edges)
  auto load = [&](const bf16* P, int T, int ld, int rows, int r0, int k0, bool drop, int c) -> bf16x8 {
    const int q = tid + 256 * c, r = r0 + (q >> 4), kk = k0 + (q & 15) * 8;
    bf16x8 v;
    const bool full = (r < rows) && (kk + 8 <= kend);
    if (T == 0 && full && ((ld & 7) == 0)) {
      v = *reinterpret_cast<const bf16x8*>(P + (size_t)r * ld + kk);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = kk + j;
        const bool ok = r < rows && k < kend;
        const size_t e = T == 0 ? (size_t)r * ld + k : (size_t)k * ld + r;
        v[j] = ok ? P[e] : (bf16)0.f;
      }
    }
    if (drop) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = kk + j;
        const unsigned long long e = T == 0 ? (unsigned long long)r * ld + k : (unsigned long long)k * ld + r;
        v[j] = (bf16)((float)v[j] * drop_scale(e, g.seed, doff, g.thresh, g.inv_keep));
      }
    }
    return v;
  };
  bf16x8 ra[CPT], rb[CPT];
  auto fetch = [&](int k0) {
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      ra[c] = load(g.A, TA, g.lda, g.M, m0, k0, DROP == 1, c);
      rb[c] = load(g.B, TB, g.ldb, g.N, n0, k0, DROP == 2, c);
    }
  };
  fetch(kbeg);
  for (int k0 = kbeg; k0 < kend; k0 += BK) {
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      const int q = tid + 256 * c, row = q >> 4, ch = q & 15;
      *reinterpret_cast<bf16x8*>(sA + row * BK + swz(row, ch) * 8) = ra[c];
      *reinterpret_cast<bf16x8*>(sB + row * BK + swz(row, ch) * 8) = rb[c];
    }
    __syncthreads();
    if (k0 + BK < kend) fetch(k0 + BK);  // block-uniform: in flight under this stage's MFMAs
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      bf16x8 af[2], bfr[2];
      const int ch = ks * 4 + (lane >> 4);  // 16x16x32: lane's k = 8 * (lane >> 4) + j of this k-step
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int r = wm * 32 + i * 16 + (lane & 15);
        af[i] = *reinterpret_cast<const bf16x8*>(sA + r * BK + swz(r, ch) * 8);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int r = wn * 32 + j * 16 + (lane & 15);
        bfr[j] = *reinterpret_cast<const bf16x8*>(sB + r * BK + swz(r, ch) * 8);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)  // C^T tile: a lane's 4 accumulators = 4 consecutive n of one m
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
  // epilogue: acc[i][j][q] = C[m = wm*32 + i*16 + (lane & 15)][n = wn*32 + j*16 + 4*(lane >> 4) + q]
  if (g.splitk > 1) {  // block-uniform: the raw partial of this split; split_gemm_reduce finishes C
    float* W = g.ws + (size_t)blockIdx.z * g.M * g.N;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int m = m0 + wm * 32 + i * 16 + (lane & 15);
      if (m >= g.M) continue;
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int n = n0 + wn * 32 + j * 16 + 4 * (lane >> 4) + q;
          if (n < g.N) W[(size_t)m * g.N + n] = acc[i][j][q];
        }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = m0 + wm * 32 + i * 16 + (lane & 15);
    if (m >= g.M) continue;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n = n0 + wn * 32 + j * 16 + 4 * (lane >> 4) + q;
        if (n >= g.N) continue;
        float v = g.alpha * acc[i][j][q];
        if (g.bias_f) v += g.bias_f[n];
        if (g.bias_h) v += (float)g.bias_h[n];
        const size_t e = (size_t)m * g.ldc + n;
        if constexpr (OUT_F32) {
          float* C = reinterpret_cast<float*>(g.C);
          C[e] = g.accumulate ? C[e] + v : v;
        } else {
          bf16* C = reinterpret_cast<bf16*>(g.C);
          C[e] = (bf16)(g.accumulate ? (float)C[e] + v : v);
        }
      }
  }
}

// split-K finish: C = alpha * (partial_0 + partial_1 + ... in split order) (+ bias) (+ C) -- the same
// fixed order for every element and every run (deterministic)
template <bool OUT_F32>
__global__ __launch_bounds__(256) void split_gemm_reduce_kernel(const GemmArgs g) {
  const long long total = (long long)g.M * g.N;
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    float s = g.ws[e];
    for (int k = 1; k < g.splitk; ++k) s += g.ws[(size_t)k * total + e];
    const int m = (int)(e / g.N), n = (int)(e - (long long)m * g.N);
    float v = g.alpha * s;
    if (g.bias_f) v += g.bias_f[n];
    if (g.bias_h) v += (float)g.bias_h[n];
    const size_t c = (size_t)m * g.ldc + n;
    if constexpr (OUT_F32) {
      float* C = reinterpret_cast<float*>(g.C);
      C[c] = g.accumulate ? C[c] + v : v;
    } else {
      bf16* C = reinterpret_cast<bf16*>(g.C);
      C[c] = (bf16)(g.accumulate ? (float)C[c] + v : v);
    }
  }
}

// db[n] (+)= sum_m X[m][n] (bf16 in, fp32 out). A workgroup owns 16 columns; its 16 row groups each
// sum every 16th row in order, then the 16 partials are added in row-group order: a fixed
// summation order (deterministic) with 16 independent chains instead of one serial pass over M.
__global__ __launch_bounds__(256) void colsum_kernel(const bf16* __restrict__ X, float* __restrict__ out, int M, int N,
                                                     int accumulate) {
  __shared__ float part[16][17];
  const int cl = threadIdx.x & 15, rg = threadIdx.x >> 4, n = blockIdx.x * 16 + cl;
  float s = 0.f;
  if (n < N)
    for (int m = rg; m < M; m += 16) s += (float)X[(size_t)m * N + n];
  part[rg][cl] = s;
  __syncthreads();
  if (rg == 0 && n < N) {
    float t = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) t += part[r][cl];
    out[n] = accumulate ? out[n] + t : t;
  }
}

// y = x * dropout-mask (the forward's h, for frozen-head training that keeps it; deterministic)
__global__ void dropout_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, long long n, unsigned long long seed,
                               unsigned offset, unsigned thresh, float inv_keep, const unsigned* offset_dev) {
  if (offset_dev) offset = *offset_dev;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    y[i] = (bf16)((float)x[i] * drop_scale((unsigned long long)i, seed, offset, thresh, inv_keep));
}

}  // namespace dbx

using namespace dbx;

template <int TA, int TB, bool F32, int DROP>
static int launch_gemm(const GemmArgs& g, hipStream_t st) {
  const int sk = g.splitk > 1 ? g.splitk : 1;
  const dim3 grid((g.N + 63) / 64, (g.M + 63) / 64, sk);
  hipLaunchKernelGGL((small_gemm_kernel<TA, TB, F32, DROP>), grid, dim3(256), 0, st, g);
  if (sk > 1) {
    const long long total = (long long)g.M * g.N;
    const int blocks = (int)((total + 255) / 256 < 1024 ? (total + 255) / 256 : 1024);
    hipLaunchKernelGGL((split_gemm_reduce_kernel<F32>), dim3(blocks), dim3(256), 0, st, g);
  }
  return (int)hipGetLastError();
}

// ta / tb: operand layouts (see above); out_f32: fp32 C (else bf16); drop: 0 / 1 (A) / 2 (B)
extern "C" int dbx_small_gemm(int ta, int tb, int out_f32, int drop, const dbx::GemmArgs* args, hipStream_t st) {
  const GemmArgs& g = *args;
  if (g.M <= 0 || g.N <= 0 || g.K <= 0) return -50;
  if (g.splitk > 1 && (g.ws == nullptr || g.splitk > 64)) return -52;
#define DBX_G(TA, TB)                                                                                   \
  if (ta == TA && tb == TB) {                                                                           \
    if (out_f32) return drop == 1 ? launch_gemm<TA, TB, true, 1>(g, st)                                 \
                        : drop == 2 ? launch_gemm<TA, TB, true, 2>(g, st) : launch_gemm<TA, TB, true, 0>(g, st); \
    return drop == 1 ? launch_gemm<TA, TB, false, 1>(g, st)                                             \
           : drop == 2 ? launch_gemm<TA, TB, false, 2>(g, st) : launch_gemm<TA, TB, false, 0>(g, st);   \
  }
  DBX_G(0, 0)
  DBX_G(0, 1)
  DBX_G(1, 1)
  DBX_G(1, 0)
#undef DBX_G
  return -51;
}

extern "C" int dbx_colsum(const bf16* X, float* out, int M, int N, int accumulate, hipStream_t st) {
  hipLaunchKernelGGL(colsum_kernel, dim3((N + 15) / 16), dim3(256), 0, st, X, out, M, N, accumulate);
  return (int)hipGetLastError();
}

extern "C" int dbx_dropout(const bf16* x, bf16* y, long long n, unsigned long long seed, unsigned offset,
                           unsigned thresh, float inv_keep, const unsigned* offset_dev, hipStream_t st) {
  long long blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(dropout_kernel, dim3((unsigned)blocks), dim3(256), 0, st, x, y, n, seed, offset, thresh, inv_keep,
                     offset_dev);
  return (int)hipGetLastError();
}
