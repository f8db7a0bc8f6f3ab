// Memory-bound CNN ops for the NHWC bf16 ResNet programs (gfx950).
//
// The reference executes these as separate MIOpen/ATen passes (BatchNorm fwd/bwd, ReLU,
// residual add, maxpool, softmax-CE, foreach optimizer: SURVEY.md §2.4 K6-K17, K20). Here each
// op is one vectorised (16 B/lane) pass, and the passes are fused where the ResNet dataflow
// allows it:
//   * BN statistics come from the conv epilogue (conv_igemm.hip); bn_finalize turns the sharded
//     partial sums into scale/shift + running stats in one tiny launch;
//   * BN-apply + residual (identity or BN'd downsample branch) + ReLU = ONE pass (bn_apply);
//   * BN backward = one reduce pass (sum g, sum g*xhat with the ReLU mask recomputed from the
//     saved pre-BN tensor or the block output) + one apply pass that writes dy (and optionally
//     the masked gradient for the residual branch) using 3 per-channel coefficients;
//   * maxpool consumes the stem's raw conv output with BN-apply+ReLU in its prologue;
//   * softmax-cross-entropy, label smoothing, argmax/correct-count and dlogits in one kernel;
//   * SGD-momentum / Adam(W) over the flat fp32 master buffer, writing the bf16 compute copy.
#include "common.h"
#include "bn_fin.h"

namespace dbx {

// ----------------------------------------------------------------------------------------
// BN finalize: stats[nshard][2][C] (fp64, see conv_igemm.hip) -> scale/shift (+ saved mean/invstd,
// running stats). Shards are summed in a fixed order, so the result is bit-reproducible.
// ----------------------------------------------------------------------------------------
// One block per 8 channels: thread (k, j) loads shard k of channel c0+j, LDS tree over the shards
// (the 32 shard loads are issued in parallel instead of as a dependent chain).
__device__ __forceinline__ void shard_sums(const double* stats, int nshard, int C, int c0, double& s_out,
                                           double& q_out, bool& active, int& c) {
  __shared__ double rs[8][33], rq[8][33];
  const int j = threadIdx.x & 7, k = threadIdx.x >> 3;  // k in 0..31
  c = c0 + j;
  double s = 0.0, q = 0.0;
  if (c < C) {
    for (int kk = k; kk < nshard; kk += 32) { s += stats[(size_t)kk * 2 * C + c]; q += stats[(size_t)kk * 2 * C + C + c]; }
  }
  rs[j][k] = s; rq[j][k] = q;
  __syncthreads();
  active = (k == 0) && (c < C);
  if (active) {
    double ss = 0.0, qq = 0.0;
    for (int t = 0; t < 32; ++t) { ss += rs[j][t]; qq += rq[j][t]; }
    s_out = ss; q_out = qq;
  }
}

__global__ void bn_finalize_kernel(const double* __restrict__ stats, int nshard, int C, float count,
                                   const float* __restrict__ gamma, const float* __restrict__ beta,
                                   float eps, float momentum, float* running_mean, float* running_var,
                                   float* scale, float* shift, float* save_mean, float* save_invstd) {
  double s = 0.0, q = 0.0;
  bool active;
  int c;
  shard_sums(stats, nshard, C, blockIdx.x * 8, s, q, active, c);
  if (!active) return;
  bn_fwd_final(c, s, q, count, gamma, beta, eps, momentum, running_mean, running_var, scale, shift, save_mean,
               save_invstd);
}

// eval-mode BN: scale/shift from running stats
__global__ void bn_eval_coeff_kernel(int C, const float* gamma, const float* beta, float eps,
                                     const float* rm, const float* rv, float* scale, float* shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float inv = rsqrtf(rv[c] + eps);
  const float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
  scale[c] = g * inv;
  shift[c] = b - rm[c] * g * inv;
}

// Channel sums of a bf16 [M][C] tensor (stats pass for layers whose producer cannot emit them)
__global__ void channel_stats_kernel(const bf16* __restrict__ y, long long M, int C, double* stats, int nshard) {
  const int tpr = C / 8, rpb = 256 / tpr;
  const int tid = threadIdx.x;
  const int cg = tid % tpr, r0 = tid / tpr;
  float s[8] = {0}, q[8] = {0};
  if (r0 < rpb) {
    for (long long m = (long long)blockIdx.x * rpb + r0; m < M; m += (long long)gridDim.x * rpb) {
      float f[8];
      unpack8(*reinterpret_cast<const u32x4*>(y + m * C + cg * 8), f);
#pragma unroll
      for (int j = 0; j < 8; ++j) { s[j] += f[j]; q[j] += f[j] * f[j]; }
    }
  }
  __shared__ float red[2][256 * 8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { red[0][tid * 8 + j] = s[j]; red[1][tid * 8 + j] = q[j]; }
  __syncthreads();
  double* st = stats + (size_t)(blockIdx.x % nshard) * 2 * C;
  for (int c = tid; c < C; c += 256) {
    const int g = c / 8, j = c % 8;
    float ss = 0.f, qq = 0.f;
    for (int r = 0; r < rpb; ++r) { ss += red[0][(r * tpr + g) * 8 + j]; qq += red[1][(r * tpr + g) * 8 + j]; }
    atomicAdd(st + c, (double)ss);
    atomicAdd(st + C + c, (double)qq);
  }
}

// ----------------------------------------------------------------------------------------
// BN apply (+ residual) (+ ReLU):  out = act(y*sc + sh + res_term)
//   RES 0: none   RES 1: + res (bf16 activation)   RES 2: + res*rsc + rsh (raw downsample conv)
// ----------------------------------------------------------------------------------------
// Thread mapping for all per-channel elementwise passes: a thread owns ONE 8-channel group
// (tpr = C/8 threads per row, rpb = 256/tpr rows per block iteration) and walks rows, so its
// per-channel coefficients are loaded once into registers instead of once per element.
struct RowMap {
  int cg, r0, rpb;
  __device__ RowMap(int C) {
    const int tpr = C >> 3;
    rpb = 256 / tpr;
    cg = threadIdx.x % tpr;
    r0 = threadIdx.x / tpr;
  }
};
__device__ __forceinline__ void load8f(const float* p, float* v) {
  const f32x4 a = *reinterpret_cast<const f32x4*>(p), b = *reinterpret_cast<const f32x4*>(p + 4);
  v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3]; v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
}

// The forward affine (scale, shift) of a thread's 8 channels: loaded (bn_finalize ran before), or
// (fin set) finalized by the block into LDS first: every thread derives a share of the C channels from
// the statistics shards (the standalone kernel's shard order and math: bit-identical); block 0 also
// stores scale / shift / saved moments / running statistics. All threads of the block must call it.
__device__ __forceinline__ void fwd_affine8(const float* sc, const float* sh, const BnFin* fin, int C, int c0,
                                            float* sk, float* s, float* h) {
  if (fin == nullptr) {
    if (c0 >= 0) { load8f(sc + c0, s); load8f(sh + c0, h); }
    return;
  }
  const BnFin& f = *fin;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    double sd = 0.0, qd = 0.0;
    for (int k = 0; k < f.nshard; ++k) {
      sd += f.stats[(size_t)k * 2 * C + c];
      qd += f.stats[(size_t)k * 2 * C + C + c];
    }
    float a, b;
    if (blockIdx.x == 0) {
      bn_fwd_final(c, sd, qd, f.count, f.gamma, f.beta, f.eps, f.momentum, f.running_mean, f.running_var, f.scale,
                   f.shift, f.mean, f.invstd);
      a = f.scale[c]; b = f.shift[c];
    } else {
      double mean, var;
      float invstd;
      bn_fwd_affine(c, sd, qd, f.count, f.gamma, f.beta, f.eps, a, b, mean, var, invstd);
    }
    sk[c] = a; sk[C + c] = b;
  }
  __syncthreads();
  if (c0 >= 0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) { s[j] = sk[c0 + j]; h[j] = sk[C + c0 + j]; }
  }
  __syncthreads();
}

template <int RES, bool RELU>
__global__ __launch_bounds__(256) void bn_apply_kernel(const bf16* __restrict__ y, const float* __restrict__ sc,
                                const float* __restrict__ sh, const bf16* __restrict__ res,
                                const float* __restrict__ rsc, const float* __restrict__ rsh,
                                bf16* __restrict__ out, unsigned char* __restrict__ mbits, long long M, int C,
                                const BnFin* __restrict__ fin, const BnFin* __restrict__ rfin) {
  __shared__ float sk[2 * 2048];
  const RowMap rm(C);
  const int c0 = rm.cg * 8, cv = rm.r0 < rm.rpb ? c0 : -1;
  float s[8], h[8], a[8], b[8];
  fwd_affine8(sc, sh, fin, C, cv, sk, s, h);
  if (RES == 2) fwd_affine8(rsc, rsh, rfin, C, cv, sk, a, b);
  if (rm.r0 >= rm.rpb) return;
  for (long long m = (long long)blockIdx.x * rm.rpb + rm.r0; m < M; m += (long long)gridDim.x * rm.rpb) {
    const long long e = m * C + c0;
    float f[8];
    unpack8(*reinterpret_cast<const u32x4*>(y + e), f);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = f[j] * s[j] + h[j];
    if (RES) {
      float r[8];
      unpack8(*reinterpret_cast<const u32x4*>(res + e), r);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] += (RES == 2) ? r[j] * a[j] + b[j] : r[j];
    }
    if (RELU) {
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = fmaxf(f[j], 0.f);
    }
    const u32x4 o = pack8(f);
    *reinterpret_cast<u32x4*>(out + e) = o;
    if (RELU && mbits) {  // 1-bit ReLU mask of the stored (bf16) values, for the backward pass
      float q[8];
      unpack8(o, q);
      unsigned bits = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) bits |= (q[j] > 0.f ? 1u : 0u) << j;
      mbits[e >> 3] = (unsigned char)bits;
    }
  }
}

// ----------------------------------------------------------------------------------------
// BN backward.
//   g = dout * mask,  MASK 0: none, 1: (mref > 0) with mref the block output,
//                     2: (y*sc + sh > 0) recomputed from the pre-BN tensor
//   reduce: sum g, sum g*xhat (xhat = (y-mean)*invstd) -> stats[nshard][2][C]
//   coeff:  dy = k1*g + k2*y + k3 ; dgamma = sum g*xhat ; dbeta = sum g
// ----------------------------------------------------------------------------------------
template <int MASK>
__device__ __forceinline__ void load_g(const bf16* dout, const bf16* mref, const bf16* y, const float* sc,
                                       const float* sh, long long e, float* g, float* yv) {
  unpack8(*reinterpret_cast<const u32x4*>(dout + e), g);
  unpack8(*reinterpret_cast<const u32x4*>(y + e), yv);
  if (MASK == 1) {
    float mr[8];
    unpack8(*reinterpret_cast<const u32x4*>(mref + e), mr);
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = mr[j] > 0.f ? g[j] : 0.f;
  } else if (MASK == 2) {
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = (yv[j] * sc[j] + sh[j]) > 0.f ? g[j] : 0.f;
  }
}

template <int MASK>
__global__ void bn_bwd_reduce_kernel(const bf16* __restrict__ dout, const bf16* __restrict__ mref,
                                     const bf16* __restrict__ y, const float* __restrict__ sc,
                                     const float* __restrict__ sh, const float* __restrict__ mean,
                                     const float* __restrict__ invstd, long long M, int C, double* stats,
                                     int nshard) {
  const int tpr = C / 8, rpb = 256 / tpr;
  const int tid = threadIdx.x;
  const int cg = tid % tpr, r0 = tid / tpr;
  const int c0 = cg * 8;
  float s[8] = {0}, q[8] = {0};
  if (r0 < rpb) {
    float mu[8], is[8], scr[8] = {0}, shr[8] = {0};
    load8f(mean + c0, mu);
    load8f(invstd + c0, is);
    if (MASK == 2) { load8f(sc + c0, scr); load8f(sh + c0, shr); }
    for (long long m = (long long)blockIdx.x * rpb + r0; m < M; m += (long long)gridDim.x * rpb) {
      float g[8], yv[8];
      load_g<MASK>(dout, mref, y, scr, shr, m * C + c0, g, yv);
#pragma unroll
      for (int j = 0; j < 8; ++j) { s[j] += g[j]; q[j] += g[j] * (yv[j] - mu[j]) * is[j]; }
    }
  }
  __shared__ float red[2][256 * 8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { red[0][tid * 8 + j] = s[j]; red[1][tid * 8 + j] = q[j]; }
  __syncthreads();
  double* st = stats + (size_t)(blockIdx.x % nshard) * 2 * C;
  for (int c = tid; c < C; c += 256) {
    const int g = c / 8, j = c % 8;
    float ss = 0.f, qq = 0.f;
    for (int r = 0; r < rpb; ++r) { ss += red[0][(r * tpr + g) * 8 + j]; qq += red[1][(r * tpr + g) * 8 + j]; }
    atomicAdd(st + c, (double)ss);
    atomicAdd(st + C + c, (double)qq);
  }
}

// per-channel backward coefficients + parameter grads (fp32, written into the flat grad buffer)
__global__ void bn_bwd_coeff_kernel(const double* __restrict__ stats, int nshard, int C, float count,
                                    const float* __restrict__ gamma, const float* __restrict__ mean,
                                    const float* __restrict__ invstd, float* coeff /*[3][C]*/,
                                    float* dgamma, float* dbeta, int accumulate) {
  double sd = 0.0, qd = 0.0;
  bool active;
  int c;
  shard_sums(stats, nshard, C, blockIdx.x * 8, sd, qd, active, c);
  if (!active) return;
  bn_bwd_final(C, c, sd, qd, count, gamma, mean, invstd, coeff, dgamma, dbeta, accumulate);
}

// The coefficients of a thread's 8 channels: loaded (bn_bwd_coeff ran before), or (fin set,
// DBX_COEFF_IN) finalized by the block into LDS first -- every thread derives a share of the C
// channels from the moment shards (bn_bwd_k's math, the standalone kernel's shard order: bit-identical;
// block 0 also stores coeff / dgamma / dbeta) -- which saves the bn_bwd_coeff launch in front of the
// apply. All threads of the block must call it (barrier inside).
__device__ __forceinline__ void bwd_coeff8(const float* coeff, const BnFin* fin, int C, int c0, float* sk, float* k1,
                                           float* k2, float* k3) {
  if (fin == nullptr) {
    if (c0 >= 0) {
      load8f(coeff + c0, k1);
      load8f(coeff + C + c0, k2);
      load8f(coeff + 2 * C + c0, k3);
    }
    return;
  }
  const BnFin& f = *fin;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    double s = 0.0, q = 0.0;
    for (int k = 0; k < f.nshard; ++k) {  // (k-ordered adds from 0.0: the standalone order)
      s += f.stats[(size_t)k * 2 * C + c];
      q += f.stats[(size_t)k * 2 * C + C + c];
    }
    float a, b, d;
    if (blockIdx.x == 0) {
      bn_bwd_final(C, c, s, q, f.count, f.gamma, f.mean, f.invstd, f.coeff, f.dgamma, f.dbeta, f.accumulate);
      a = f.coeff[c]; b = f.coeff[C + c]; d = f.coeff[2 * C + c];
    } else {
      bn_bwd_k(s, q, f.count, f.gamma ? f.gamma[c] : 1.f, f.invstd[c], f.mean[c], a, b, d);
    }
    sk[c] = a; sk[C + c] = b; sk[2 * C + c] = d;
  }
  __syncthreads();
  if (c0 >= 0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) { k1[j] = sk[c0 + j]; k2[j] = sk[C + c0 + j]; k3[j] = sk[2 * C + c0 + j]; }
  }
  __syncthreads();  // (sk reusable by a second call)
}

template <int MASK, bool WRITE_G>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const bf16* __restrict__ dout, const bf16* __restrict__ mref,
                                    const bf16* __restrict__ y, const float* __restrict__ sc,
                                    const float* __restrict__ sh, const float* __restrict__ coeff,
                                    bf16* __restrict__ dy, bf16* __restrict__ gout, long long M, int C,
                                    const BnFin* __restrict__ fin) {
  __shared__ float sk[3 * 2048];
  const RowMap rm(C);
  const int c0 = rm.cg * 8;
  float k1[8], k2[8], k3[8], scr[8] = {0}, shr[8] = {0};
  bwd_coeff8(coeff, fin, C, rm.r0 < rm.rpb ? c0 : -1, sk, k1, k2, k3);
  if (rm.r0 >= rm.rpb) return;
  if (MASK == 2) { load8f(sc + c0, scr); load8f(sh + c0, shr); }
  for (long long m = (long long)blockIdx.x * rm.rpb + rm.r0; m < M; m += (long long)gridDim.x * rm.rpb) {
    const long long e = m * C + c0;
    float g[8], yv[8];
    load_g<MASK>(dout, mref, y, scr, shr, e, g, yv);
    if (WRITE_G) *reinterpret_cast<u32x4*>(gout + e) = pack8(g);
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = k1[j] * g[j] + k2[j] * yv[j] + k3[j];
    *reinterpret_cast<u32x4*>(dy + e) = pack8(o);
  }
}

// Two BN backward applies fed by the same gradient (the block tail of a downsample block:
// bn3 of the main branch and the downsample BN): g is read once for both outputs.
__global__ __launch_bounds__(256) void bn_bwd_apply2_kernel(const bf16* __restrict__ g_in, const bf16* __restrict__ y1,
                                                            const float* __restrict__ coeff1, bf16* __restrict__ dy1,
                                                            const bf16* __restrict__ y2, const float* __restrict__ coeff2,
                                                            bf16* __restrict__ dy2, long long M, int C,
                                                            const BnFin* __restrict__ fin1, const BnFin* __restrict__ fin2) {
  __shared__ float sk[3 * 2048];
  const RowMap rm(C);
  const int c0 = rm.cg * 8, cv = rm.r0 < rm.rpb ? c0 : -1;
  float a1[8], a2[8], a3[8], b1[8], b2[8], b3[8];
  bwd_coeff8(coeff1, fin1, C, cv, sk, a1, a2, a3);
  bwd_coeff8(coeff2, fin2, C, cv, sk, b1, b2, b3);
  if (rm.r0 >= rm.rpb) return;
  for (long long m = (long long)blockIdx.x * rm.rpb + rm.r0; m < M; m += (long long)gridDim.x * rm.rpb) {
    const long long e = m * C + c0;
    float g[8], u[8], v[8], o1[8], o2[8];
    unpack8(*reinterpret_cast<const u32x4*>(g_in + e), g);
    unpack8(*reinterpret_cast<const u32x4*>(y1 + e), u);
    unpack8(*reinterpret_cast<const u32x4*>(y2 + e), v);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      o1[j] = a1[j] * g[j] + a2[j] * u[j] + a3[j];
      o2[j] = b1[j] * g[j] + b2[j] * v[j] + b3[j];
    }
    *reinterpret_cast<u32x4*>(dy1 + e) = pack8(o1);
    *reinterpret_cast<u32x4*>(dy2 + e) = pack8(o2);
  }
}

// ----------------------------------------------------------------------------------------
// MaxPool 3x3 s2 p1 (NHWC) with BN-apply + ReLU prologue; argmax (0..8) saved as uint8.
// ----------------------------------------------------------------------------------------
// KF > 0: the window size as a constant (the ResNet stem's 3x3 / stride-2 pool) -- all KF x KF loads
// of a window issued before any compare (out-of-image taps masked, no branches between the loads) and
// 32-bit pixel arithmetic (host-checked M < 2^31); the compares run in the generic path's (r, s) order
// with the same strict '>', so the argmax (and its ties) are identical.
template <int KF>
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(const bf16* __restrict__ x, const float* __restrict__ sc,
                                   const float* __restrict__ sh, bf16* __restrict__ out,
                                   unsigned char* __restrict__ arg, bf16* __restrict__ ymax, int N, int H, int W,
                                   int C, int P, int Q, int K, int stride, int pad, int relu,
                                   const BnFin* __restrict__ fin) {
  __shared__ float sk[2 * 2048];
  const RowMap rm(C);
  const int c0 = rm.cg * 8;
  float s[8], h[8];
  if (fin) fwd_affine8(sc, sh, fin, C, rm.r0 < rm.rpb ? c0 : -1, sk, s, h);  // (the stem BN finalized here)
  if (rm.r0 >= rm.rpb) return;
  if (fin) {
  } else if (sc) { load8f(sc + c0, s); load8f(sh + c0, h); }
  else {
#pragma unroll
    for (int j = 0; j < 8; ++j) { s[j] = 1.f; h[j] = 0.f; }
  }
  const long long M = (long long)N * P * Q;
  for (long long pix = (long long)blockIdx.x * rm.rpb + rm.r0; pix < M; pix += (long long)gridDim.x * rm.rpb) {
    int q, p, n;
    if constexpr (KF > 0) {
      const int pi = (int)pix, t = pi / Q;
      q = pi - t * Q; n = t / P; p = t - n * P;
    } else {
      q = (int)(pix % Q);
      const long long t = pix / Q;
      p = (int)(t % P);
      n = (int)(t / P);
    }
    float best[8], braw[8];
    unsigned char bi[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; braw[j] = 0.f; bi[j] = 0; }
    if constexpr (KF > 0) {
      u32x4 win[KF * KF];
      bool ok[KF * KF];
#pragma unroll
      for (int r = 0; r < KF; ++r)
#pragma unroll
        for (int ss = 0; ss < KF; ++ss) {
          const int hh = p * stride - pad + r, w = q * stride - pad + ss;
          const bool v = (unsigned)hh < (unsigned)H && (unsigned)w < (unsigned)W;
          ok[r * KF + ss] = v;
          win[r * KF + ss] = *reinterpret_cast<const u32x4*>(
              x + (((size_t)n * H + (v ? hh : 0)) * W + (v ? w : 0)) * C + c0);
        }
#pragma unroll
      for (int k = 0; k < KF * KF; ++k) {
        float f[8];
        unpack8(win[k], f);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float v = f[j] * s[j] + h[j];
          if (relu) v = fmaxf(v, 0.f);
          if (ok[k] && v > best[j]) { best[j] = v; braw[j] = f[j]; bi[j] = (unsigned char)k; }
        }
      }
    }
    for (int r = 0; r < (KF > 0 ? 0 : K); ++r) {
      const int hh = p * stride - pad + r;
      if (hh < 0 || hh >= H) continue;
      for (int ss = 0; ss < K; ++ss) {
        const int w = q * stride - pad + ss;
        if (w < 0 || w >= W) continue;
        float f[8];
        unpack8(*reinterpret_cast<const u32x4*>(x + (((size_t)n * H + hh) * W + w) * C + c0), f);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float v = f[j] * s[j] + h[j];
          if (relu) v = fmaxf(v, 0.f);
          if (v > best[j]) { best[j] = v; braw[j] = f[j]; bi[j] = (unsigned char)(r * K + ss); }
        }
      }
    }
    const size_t o = (size_t)pix * C + c0;
    *reinterpret_cast<u32x4*>(out + o) = pack8(best);
    *reinterpret_cast<uint2*>(arg + o) = *reinterpret_cast<uint2*>(bi);
    // the pre-BN value at the argmax: the stem BN-backward reduction then runs over the pooled
    // positions (sum over windows == sum over pixels of the scattered gradient), 1/4 of the bytes
    if (ymax) *reinterpret_cast<u32x4*>(ymax + o) = pack8(braw);
  }
}

// gather form of the backward (no atomics): dx[n,h,w,c] = sum over windows whose argmax is (h,w)
__global__ void maxpool_bwd_kernel(const bf16* __restrict__ dout, const unsigned char* __restrict__ arg,
                                   bf16* __restrict__ dx, int N, int H, int W, int C, int P, int Q, int K,
                                   int stride, int pad) {
  const int cpt = C / 8;
  const long long total = (long long)N * H * W * cpt;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int cg = (int)(i % cpt);
    long long pix = i / cpt;
    const int w = (int)(pix % W); pix /= W;
    const int h = (int)(pix % H);
    const int n = (int)(pix / H);
    const int c0 = cg * 8;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // outputs p with p*stride - pad <= h <= p*stride - pad + K - 1
    const int p_lo = max(0, (h + pad - K + stride) / stride), p_hi = min(P - 1, (h + pad) / stride);
    const int q_lo = max(0, (w + pad - K + stride) / stride), q_hi = min(Q - 1, (w + pad) / stride);
    for (int p = p_lo; p <= p_hi; ++p) {
      const int r = h - (p * stride - pad);
      if (r < 0 || r >= K) continue;
      for (int q = q_lo; q <= q_hi; ++q) {
        const int s = w - (q * stride - pad);
        if (s < 0 || s >= K) continue;
        const size_t o = (((size_t)n * P + p) * Q + q) * C + c0;
        float g[8];
        unpack8(*reinterpret_cast<const u32x4*>(dout + o), g);
        const uint2 av = *reinterpret_cast<const uint2*>(arg + o);
        const unsigned char* a8 = reinterpret_cast<const unsigned char*>(&av);
        const unsigned char me = (unsigned char)(r * K + s);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += (a8[j] == me) ? g[j] : 0.f;
      }
    }
    *reinterpret_cast<u32x4*>(dx + (((size_t)n * H + h) * W + w) * C + c0) = pack8(acc);
  }
}

// ----------------------------------------------------------------------------------------
// Stem backward without the pooled-gradient tensor: the max-pool backward (gather form) is
// recomputed inside the BN-backward reduce and apply passes of the stem BN, so the [N,112,112,64]
// gradient of the pool input is never written or re-read (3 x 1.6 GB at batch 1024).
//   g[n,h,w,c] = sum over pool windows (p,q) containing (h,w) with argmax == (h,w): dpool[n,p,q,c]
//   g *= (y*sc + sh > 0)                       (the ReLU between the stem BN and the pool)
//   reduce: stats += [sum g, sum g*xhat]       apply: dy = k1*g + k2*y + k3
// A block walks whole image rows (n, h): the window rows p are block-uniform, and at most two
// windows per dimension contain a pixel (host-checked: ceil(K/stride) <= 2), so the gather is a
// fixed 2x2 candidate set with clamped addresses and selects (no branches around loads).
// 32-bit offsets: host checks N*H*W*C < 2^31.
// ----------------------------------------------------------------------------------------
template <bool APPLY>
__global__ __launch_bounds__(256) void pool_bn_bwd_kernel(const bf16* __restrict__ dpool,
                                                          const unsigned char* __restrict__ arg,
                                                          const bf16* __restrict__ y, const float* __restrict__ sc,
                                                          const float* __restrict__ sh, const float* __restrict__ c1,
                                                          const float* __restrict__ c2, const float* __restrict__ c3,
                                                          bf16* __restrict__ dy, double* __restrict__ stats, int nshard,
                                                          int N, int H, int W, int C, int P, int Q, int K, int stride,
                                                          int pad) {
  const int cpt = C >> 3;  // 256 % cpt == 0 (host): a thread's channel group is fixed
  const int tid = threadIdx.x;
  const int c0 = (tid % cpt) * 8;
  float s_[8], h_[8], k1[8], k2[8], k3[8];
  load8f(sc + c0, s_);
  load8f(sh + c0, h_);
  load8f(c1 + c0, k1);  // reduce: mean, invstd ; apply: k1, k2, k3
  load8f(c2 + c0, k2);
  if (APPLY) load8f(c3 + c0, k3);
  float as[8] = {0, 0, 0, 0, 0, 0, 0, 0}, aq[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int rows = N * H, per_row = W * cpt;
  for (int row = blockIdx.x; row < rows; row += gridDim.x) {
    const int n = row / H, h = row - n * H;
    const int p_lo = max(0, (h + pad - K + stride) / stride), p_hi = min(P - 1, (h + pad) / stride);
    const int r_lo = h + pad - p_lo * stride;
    const bool p1 = p_hi >= p_lo, p2 = p_hi > p_lo;  // block-uniform: first / second window row exist
    const int pc = p1 ? p_lo : 0;
    const int prow0 = (n * P + pc) * Q, prow1 = (n * P + (p2 ? p_lo + 1 : pc)) * Q;
    for (int i = tid; i < per_row; i += 256) {
      const int w = i / cpt;
      const int q_lo = max(0, (w + pad - K + stride) / stride);
      u32x4 gd[2][2];
      uint2 av[2][2];
      bool ok[2][2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int q = q_lo + t;
        const int s = w + pad - q * stride;
        const bool vq = q < Q && s >= 0 && s < K;
        const int qq = vq ? q : 0;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int o = ((u ? prow1 : prow0) + qq) * C + c0;
          gd[u][t] = *reinterpret_cast<const u32x4*>(dpool + o);
          av[u][t] = *reinterpret_cast<const uint2*>(arg + o);
          ok[u][t] = vq && (u == 0 ? p1 : p2);
        }
      }
      const int e = (row * W + w) * C + c0;
      float yv[8];
      unpack8(*reinterpret_cast<const u32x4*>(y + e), yv);
      float g[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int r = r_lo - u * stride, s = w + pad - (q_lo + t) * stride;
          const unsigned me = (unsigned)(r * K + s);
          float gv[8];
          unpack8(gd[u][t], gv);
          const unsigned char* a8 = reinterpret_cast<const unsigned char*>(&av[u][t]);
#pragma unroll
          for (int j = 0; j < 8; ++j) g[j] += (ok[u][t] && a8[j] == me) ? gv[j] : 0.f;
        }
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = (yv[j] * s_[j] + h_[j]) > 0.f ? g[j] : 0.f;
      if (APPLY) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = k1[j] * g[j] + k2[j] * yv[j] + k3[j];
        *reinterpret_cast<u32x4*>(dy + e) = pack8(o);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) { as[j] += g[j]; aq[j] += g[j] * (yv[j] - k1[j]) * k2[j]; }
      }
    }
  }
  if (!APPLY) {
    __shared__ float red[2][256 * 8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { red[0][tid * 8 + j] = as[j]; red[1][tid * 8 + j] = aq[j]; }
    __syncthreads();
    double* st = stats + (size_t)(blockIdx.x % nshard) * 2 * C;
    for (int c = tid; c < C; c += 256) {
      const int gi = c / 8, j = c % 8;
      float ss = 0.f, qq = 0.f;
      for (int r = 0; r < 256 / cpt; ++r) { ss += red[0][(r * cpt + gi) * 8 + j]; qq += red[1][(r * cpt + gi) * 8 + j]; }
      atomicAdd(st + c, (double)ss);
      atomicAdd(st + C + c, (double)qq);
    }
  }
}

// ----------------------------------------------------------------------------------------
// Global average pool [N][HW][C] -> [N][C] (bf16 out, fp32 accumulate) and its backward
// ----------------------------------------------------------------------------------------
__global__ void avgpool_fwd_kernel(const bf16* __restrict__ x, bf16* __restrict__ out, int N, int HW, int C) {
  const int n = blockIdx.y;
  const int c0 = (blockIdx.x * blockDim.x + threadIdx.x) * 8;
  if (c0 >= C) return;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < HW; ++i) {
    float f[8];
    unpack8(*reinterpret_cast<const u32x4*>(x + ((size_t)n * HW + i) * C + c0), f);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += f[j];
  }
  const float inv = 1.f / HW;
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] *= inv;
  *reinterpret_cast<u32x4*>(out + (size_t)n * C + c0) = pack8(acc);
}

__global__ void avgpool_bwd_kernel(const bf16* __restrict__ dout, bf16* __restrict__ dx, int N, int HW, int C) {
  const long long total = (long long)N * HW * C / 8;
  const float inv = 1.f / HW;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const long long e = i * 8;
    const int c0 = (int)(e % C);
    const long long n = e / ((long long)HW * C);
    float f[8];
    unpack8(*reinterpret_cast<const u32x4*>(dout + n * C + c0), f);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] *= inv;
    *reinterpret_cast<u32x4*>(dx + e) = pack8(f);
  }
}

// ----------------------------------------------------------------------------------------
// Softmax cross-entropy (+label smoothing) fused with dlogits, argmax-correct count.
// One 256-thread block per row; logits fp32 or bf16; dlogits = (p - target)/B * gscale.
// out_stats[0] += sum loss, out_stats[1] += correct   (fp64 device accumulators: no host sync,
// order-independent sums)
// ----------------------------------------------------------------------------------------
template <typename T>
__global__ void softmax_ce_kernel(const T* __restrict__ logits, const long long* __restrict__ labels,
                                  T* __restrict__ dlogits, float* __restrict__ loss_out, double* stats,
                                  int B, int C, float smoothing, float gscale,
                                  const long long* __restrict__ labels2, const float* __restrict__ lam_ptr) {
  // labels2 / lam_ptr (CutMix): target = lam * onehot(label) + (1 - lam) * onehot(label2), then label
  // smoothing on top (Composer applies LabelSmoothing to the mixed targets); accuracy vs label
  const int row = blockIdx.x;
  const T* x = logits + (size_t)row * C;
  const int tid = threadIdx.x;
  __shared__ float red[8];
  __shared__ int redi[8];
  float mx = -INFINITY;
  int amx = 0;
  for (int c = tid; c < C; c += 256) {
    const float v = (float)x[c];
    if (v > mx) { mx = v; amx = c; }
  }
  // argmax-aware max reduction
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(mx, o, 64);
    const int oa = __shfl_xor(amx, o, 64);
    if (om > mx || (om == mx && oa < amx)) { mx = om; amx = oa; }
  }
  const int wid = tid >> 6, lane = tid & 63;
  if (lane == 0) { red[wid] = mx; redi[wid] = amx; }
  __syncthreads();
  if (tid == 0) {
    for (int w = 1; w < 4; ++w)
      if (red[w] > red[0] || (red[w] == red[0] && redi[w] < redi[0])) { red[0] = red[w]; redi[0] = redi[w]; }
  }
  __syncthreads();
  mx = red[0];
  amx = redi[0];
  __syncthreads();
  float se = 0.f, sx = 0.f;
  for (int c = tid; c < C; c += 256) {
    const float v = (float)x[c];
    se += __expf(v - mx);
    sx += v;
  }
  se = wave_sum(se);
  sx = wave_sum(sx);
  if (lane == 0) { red[wid] = se; red[4 + wid] = sx; }
  __syncthreads();
  se = red[0] + red[1] + red[2] + red[3];
  sx = red[4] + red[5] + red[6] + red[7];
  const float lse = mx + __logf(se);
  const long long lab = labels[row];
  const float xl = (float)x[lab];
  const float lam = labels2 ? lam_ptr[0] : 1.f;
  const long long lab2 = labels2 ? labels2[row] : lab;
  const float xl2 = (float)x[lab2];
  // loss = -(1-eps) * [lam log p_lab + (1-lam) log p_lab2] - eps/C * sum_c log p_c
  const float loss = (1.f - smoothing) * (lam * (lse - xl) + (1.f - lam) * (lse - xl2)) + smoothing * (lse - sx / C);
  if (tid == 0) {
    if (loss_out) loss_out[row] = loss;
    if (stats) {
      atomicAdd(stats, (double)loss);
      atomicAdd(stats + 1, (amx == lab) ? 1.0 : 0.0);
    }
  }
  if (dlogits) {
    const float inv = gscale / B;
    for (int c = tid; c < C; c += 256) {
      const float p = __expf((float)x[c] - lse);
      const float t = (1.f - smoothing) * ((c == lab ? lam : 0.f) + (c == lab2 ? 1.f - lam : 0.f)) + smoothing / C;
      dlogits[(size_t)row * C + c] = (T)((p - t) * inv);
    }
  }
}

// ----------------------------------------------------------------------------------------
// Fused optimizers over the flat fp32 master buffer (+ optional bf16 compute copy).
//   SGD (PyTorch semantics): d = g + wd*p; v = mom*v + (1-damp)*d (v = d at step 1);
//                            d = nesterov ? d + mom*v : v; p -= lr*d
//   Adam/AdamW: m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2; p -= lr * mhat/(sqrt(vhat)+eps)
//   grad_scale multiplies g first (DDP averaging / loss scaling / clipping factor), read
//   from device memory so it can be produced by a previous kernel (global-norm clip).
// ----------------------------------------------------------------------------------------
__global__ void sgd_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ v,
                           bf16* __restrict__ p16, long long n, const float* __restrict__ hyper, float lr, float mom,
                           float damp, float wd, int nesterov, int first, const float* __restrict__ gscale_ptr,
                           float gscale) {
  // hyper (device, nullable): [lr] so a captured graph follows the LR schedule on replay
  if (hyper) lr = hyper[0];
  const float gs = gscale_ptr ? gscale * gscale_ptr[0] : gscale;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i * 4 < n; i += (long long)gridDim.x * blockDim.x) {
    const long long e = i * 4;
    if (e + 4 <= n) {
      f32x4 pp = *reinterpret_cast<f32x4*>(p + e);
      f32x4 gg = *reinterpret_cast<const f32x4*>(g + e) * gs;
      gg += wd * pp;
      f32x4 d = gg;
      if (mom != 0.f) {
        f32x4 vv = first ? gg : (*reinterpret_cast<f32x4*>(v + e) * mom + (1.f - damp) * gg);
        *reinterpret_cast<f32x4*>(v + e) = vv;
        d = nesterov ? gg + mom * vv : vv;
      }
      pp -= lr * d;
      *reinterpret_cast<f32x4*>(p + e) = pp;
      if (p16) {
        bf16x4 b = {(bf16)pp[0], (bf16)pp[1], (bf16)pp[2], (bf16)pp[3]};
        *reinterpret_cast<bf16x4*>(p16 + e) = b;
      }
    } else {
      for (long long k = e; k < n; ++k) {
        float gg = g[k] * gs + wd * p[k];
        float d = gg;
        if (mom != 0.f) {
          const float vv = first ? gg : v[k] * mom + (1.f - damp) * gg;
          v[k] = vv;
          d = nesterov ? gg + mom * vv : vv;
        }
        p[k] -= lr * d;
        if (p16) p16[k] = (bf16)p[k];
      }
    }
  }
}

// ----------------------------------------------------------------------------------------
// LARS (layer-wise adaptive rate scaling, large-batch SGD): per parameter tensor ("segment")
//   trust = eta * |w| / (|g| + wd * |w|)      (1 when either norm is 0)
//   g    <- adapt ? trust * (gs * g + wd * w) : gs * g
// followed by the plain SGD kernel with wd = 0. grid = (chunks, nseg): blockIdx.y is the segment,
// blocks stride over it; phase 1 reduces |w|^2 and |gs*g|^2 per segment (wave shuffles, one LDS
// step over the 4 waves) into one fp64 partial pair per (segment, block) slot -- no atomics; phase 2
// sums a segment's partials in block order (every block the same fixed order), so the trust ratios
// are bit-reproducible whatever order the blocks ran in, then rescales in place.
// ----------------------------------------------------------------------------------------
constexpr int kLarsMaxBlocks = 64;  // blocks per segment (dbx_lars_scale clamps to this)
__global__ void lars_norms_kernel(const float* __restrict__ p, const float* __restrict__ g,
                                  const int* __restrict__ seg_off, const int* __restrict__ seg_len, float gs,
                                  double* __restrict__ norms) {
  const int s = blockIdx.y;
  const int off = seg_off[s], len = seg_len[s];
  float ww = 0.f, gg = 0.f;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < len; i += gridDim.x * blockDim.x) {
    const float w = p[off + i], d = g[off + i] * gs;
    ww += w * w;
    gg += d * d;
  }
  for (int o = 32; o > 0; o >>= 1) {
    ww += __shfl_xor(ww, o, 64);
    gg += __shfl_xor(gg, o, 64);
  }
  __shared__ float red[2][4];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) {
    red[0][wave] = ww;
    red[1][wave] = gg;
  }
  __syncthreads();
  if (threadIdx.x == 0) {  // slot (s, block): norms is [nseg][kLarsMaxBlocks][2]
    double* o = norms + 2 * ((size_t)s * kLarsMaxBlocks + blockIdx.x);
    o[0] = (double)(red[0][0] + red[0][1] + red[0][2] + red[0][3]);
    o[1] = (double)(red[1][0] + red[1][1] + red[1][2] + red[1][3]);
  }
}

__global__ void lars_apply_kernel(const float* __restrict__ p, float* __restrict__ g, const int* __restrict__ seg_off,
                                  const int* __restrict__ seg_len, const int* __restrict__ adapt,
                                  const double* __restrict__ norms, float gs, float eta, float wd) {
  const int s = blockIdx.y;
  const int off = seg_off[s], len = seg_len[s];
  float scale = gs, decay = 0.f;
  if (adapt[s]) {
    double ww = 0.0, gg = 0.0;  // fixed block order (gridDim.x slots written by lars_norms_kernel)
    const double* o = norms + 2 * (size_t)s * kLarsMaxBlocks;
    for (int b = 0; b < (int)gridDim.x; ++b) { ww += o[2 * b]; gg += o[2 * b + 1]; }
    const float wn = (float)sqrt(ww), gn = (float)sqrt(gg);
    const float trust = (wn > 0.f && gn > 0.f) ? eta * wn / (gn + wd * wn) : 1.f;
    scale = trust * gs;
    decay = trust * wd;
  }
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < len; i += gridDim.x * blockDim.x)
    g[off + i] = scale * g[off + i] + decay * p[off + i];
}

__global__ void adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, bf16* __restrict__ p16, long long n, const float* __restrict__ hyper,
                            float lr, float b1, float b2, float eps, float wd, int decoupled, float bc1, float bc2,
                            const float* __restrict__ gscale_ptr, float gscale) {
  // hyper (device, nullable): [lr, 1-b1^t, 1-b2^t] so graph replays track the step count
  if (hyper) { lr = hyper[0]; bc1 = hyper[1]; bc2 = hyper[2]; }
  const float gs = gscale_ptr ? gscale * gscale_ptr[0] : gscale;
  for (long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (long long)gridDim.x * blockDim.x) {
    float gg = g[k] * gs;
    float pp = p[k];
    if (decoupled) pp -= lr * wd * pp;
    else gg += wd * pp;
    const float mm = b1 * m[k] + (1.f - b1) * gg;
    const float vv = b2 * v[k] + (1.f - b2) * gg * gg;
    m[k] = mm; v[k] = vv;
    pp -= lr * (mm / bc1) / (sqrtf(vv / bc2) + eps);
    p[k] = pp;
    if (p16) p16[k] = (bf16)pp;
  }
}

// sum of squares over a flat fp32 buffer (global-norm clipping), one fp64 atomic per block. fp64
// sums of fp32 block partials are exact (hence independent of block order) while the partials'
// magnitudes span less than ~2^29; beyond that the last bits of the norm can depend on the order.
__global__ void sumsq_kernel(const float* __restrict__ x, long long n, double* out) {
  float s = 0.f;
  for (long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (long long)gridDim.x * blockDim.x) s += x[k] * x[k];
  s = wave_sum(s);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(out, (double)(red[0] + red[1] + red[2] + red[3]));
}

// clip factor = min(1, max_norm / (sqrt(sumsq) + 1e-6)) written to out[0]
__global__ void clip_factor_kernel(const double* sumsq, float max_norm, float* out) {
  const float nrm = (float)sqrt(sumsq[0]);
  out[0] = fminf(1.f, max_norm / (nrm + 1e-6f));
  out[1] = nrm;
}

// ----------------------------------------------------------------------------------------
// Input: uint8 NHWC [N][H][W][3] -> bf16 NHWC4 normalised ((x/255 - mean)/std, ch3 = 0),
// optional per-sample horizontal flip (flags[n] != 0).
// ----------------------------------------------------------------------------------------
__global__ void normalize_u8_kernel(const unsigned char* __restrict__ in, bf16* __restrict__ out,
                                    const unsigned char* __restrict__ flip, int N, int H, int W, int Cin,
                                    float m0, float m1, float m2, float s0, float s1, float s2) {
  const long long total = (long long)N * H * W;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int w = (int)(i % W);
    const long long nh = i / W;
    const int n = (int)(nh / H);
    const int ws = (flip && flip[n]) ? (W - 1 - w) : w;
    const unsigned char* src = in + ((nh * W) + ws) * Cin;
    float f0, f1, f2;
    if (Cin == 1) { f0 = f1 = f2 = src[0] * (1.f / 255.f); }
    else { f0 = src[0] * (1.f / 255.f); f1 = src[1] * (1.f / 255.f); f2 = src[2] * (1.f / 255.f); }
    bf16x4 o = {(bf16)((f0 - m0) / s0), (bf16)((f1 - m1) / s1), (bf16)((f2 - m2) / s2), (bf16)0.f};
    *reinterpret_cast<bf16x4*>(out + i * 4) = o;
  }
}

// ----------------------------------------------------------------------------------------
// GPU input augmentation: uint8 NHWC [N][Hin][Win][Cin] -> bf16 NHWC4
// [N][Ho][Wo][4]: per-sample crop box (y0, x0, h, w in source pixels, float) resized to Ho x Wo
// with bilinear sampling (pixel-centre convention, edge clamp), optional horizontal flip,
// (x/255 - mean)/std, channel 3 = 0. Covers RandomResizedCrop / RandomCrop(pad) / Resize /
// CenterCrop + RandomHorizontalFlip + Normalize of the reference's CPU transform chains.
// ----------------------------------------------------------------------------------------
// One block per output row (n, oy): the box, flip and the two source rows are block-uniform, so
// per pixel only the column interpolation is computed (32-bit index math throughout).
// CutMix (Composer's CutMix(alpha=1), `03_composer/01_cifar_composer_resnet.ipynb:430`):
// with perm / mixbox set, output pixels inside the batch-wide box [y0, y1) x [x0, x1) come from
// sample perm[n] -- sampled with ITS crop box and flip, i.e. exactly the pixels of the augmented
// image perm[n] at the same output position (Composer pastes after the per-sample transforms).
__global__ __launch_bounds__(256) void augment_u8_kernel(const unsigned char* __restrict__ in, bf16* __restrict__ out,
                                                         const float* __restrict__ boxes,
                                                         const unsigned char* __restrict__ flip, int N, int Hin,
                                                         int Win, int Cin, int Ho, int Wo, float m0, float m1,
                                                         float m2, float s0, float s1, float s2,
                                                         const int* __restrict__ perm, const int* __restrict__ mixbox) {
  constexpr int kRowMax = 4096;
  __shared__ __attribute__((aligned(16))) unsigned char srow[2][kRowMax];
  const int my0 = mixbox ? mixbox[0] : 0, my1 = mixbox ? mixbox[1] : 0;
  const int mx0 = mixbox ? mixbox[2] : 0, mx1 = mixbox ? mixbox[3] : 0;
  const float i0 = 1.f / (255.f * s0), i1 = 1.f / (255.f * s1), i2 = 1.f / (255.f * s2);
  for (int row = blockIdx.x; row < N * Ho; row += gridDim.x) {  // row = n * Ho + oy
  const int n = row / Ho, oy = row - n * Ho;
  const bool mixrow = perm && oy >= my0 && oy < my1 && mx0 < mx1;  // block-uniform
  // pass 0: sample n outside the box (everywhere when not mixing); pass 1: sample perm[n] inside
  for (int pass = 0; pass < (mixrow ? 2 : 1); ++pass) {
  const int sn = pass ? perm[n] : n;
  const int xlo = pass ? mx0 : 0, xhi = pass ? mx1 : Wo;
  const float by = boxes[4 * sn], bx = boxes[4 * sn + 1], bh = boxes[4 * sn + 2], bw = boxes[4 * sn + 3];
  const bool fl = flip && flip[sn];
  float sy = by + (oy + 0.5f) * bh / Ho - 0.5f;
  sy = fminf(fmaxf(sy, 0.f), (float)(Hin - 1));
  const int y0 = (int)sy, y1 = min(y0 + 1, Hin - 1);
  const float wy = sy - y0;
  const unsigned char* g0 = in + ((size_t)sn * Hin + y0) * Win * Cin;
  const unsigned char* g1 = in + ((size_t)sn * Hin + y1) * Win * Cin;
  // the two source rows are staged in LDS with 16-byte loads (the bilinear taps are byte gathers)
  const int rb = Win * Cin;
  const bool staged = rb <= kRowMax && (((size_t)g0 | (size_t)g1) & 15) == 0 && (rb & 15) == 0;  // block-uniform
  if (staged) {
    for (int o = threadIdx.x * 16; o < rb; o += blockDim.x * 16) {
      *reinterpret_cast<u32x4*>(&srow[0][o]) = *reinterpret_cast<const u32x4*>(g0 + o);
      *reinterpret_cast<u32x4*>(&srow[1][o]) = *reinterpret_cast<const u32x4*>(g1 + o);
    }
    __syncthreads();
  }
  const float sxs = bw / Wo;
  auto body = [&](const unsigned char* r0, const unsigned char* r1) __attribute__((always_inline)) {
    for (int ox = xlo + threadIdx.x; ox < xhi; ox += blockDim.x) {
      if (mixrow && !pass && ox >= mx0 && ox < mx1) continue;  // pasted by pass 1
      const int oxx = fl ? (Wo - 1 - ox) : ox;
      float sx = bx + (oxx + 0.5f) * sxs - 0.5f;
      sx = fminf(fmaxf(sx, 0.f), (float)(Win - 1));
      const int x0 = (int)sx, x1 = min(x0 + 1, Win - 1);
      const float wx = sx - x0;
      float v[3];
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const int cc = Cin == 1 ? 0 : c;
        const float a = r0[x0 * Cin + cc], b = r0[x1 * Cin + cc];
        const float d = r1[x0 * Cin + cc], e = r1[x1 * Cin + cc];
        v[c] = (a * (1.f - wx) + b * wx) * (1.f - wy) + (d * (1.f - wx) + e * wx) * wy;  // 0..255
      }
      bf16x4 o = {(bf16)(v[0] * i0 - m0 / s0), (bf16)(v[1] * i1 - m1 / s1), (bf16)(v[2] * i2 - m2 / s2), (bf16)0.f};
      *reinterpret_cast<bf16x4*>(out + ((size_t)row * Wo + ox) * 4) = o;
    }
  };
  if (staged) body(&srow[0][0], &srow[1][0]);  // LDS byte gathers (ds_read_u8)
  else body(g0, g1);
  __syncthreads();  // srow reuse by the next pass / row
  }
  }
}

// ----------------------------------------------------------------------------------------
// Weight prep: fp32 KRSC master -> bf16 KRSC (fwd) and bf16 CRSK (dgrad) ; batched over layers
// ----------------------------------------------------------------------------------------
struct WDesc { long long src, fwd, tr; int K, RS, C, pad; };
// blockIdx.y = layer. Layers with a dgrad copy (K, C multiples of 64) are processed in 64x64
// (k, c) tiles per tap through LDS so both the KRSC and the transposed CRSK stores are
// coalesced; the others (fc) are a plain vectorised cast.
// 4 consecutive source elements (fp32 master or, under ZeRO, the all-gathered bf16 copy) as bf16
__device__ __forceinline__ bf16x4 load4_bf16(const float* p) {
  const float4 v = *reinterpret_cast<const float4*>(p);
  return bf16x4{(bf16)v.x, (bf16)v.y, (bf16)v.z, (bf16)v.w};
}
__device__ __forceinline__ bf16x4 load4_bf16(const bf16* p) { return *reinterpret_cast<const bf16x4*>(p); }

template <typename T>
__global__ __launch_bounds__(256) void weight_prep_kernel(const T* __restrict__ master, bf16* __restrict__ wbuf,
                                                          const WDesc* __restrict__ desc, int nlayers) {
  const WDesc d = desc[blockIdx.y];
  const int tid = threadIdx.x;
  // per-step utility work folded into this launch (one graph node instead of four):
  //   tr == -2: the stem weight (K, R, S, C) at d.src -> bf16 (K, 8, 8, 4) at d.fwd, zero padded
  //             (R = d.RS >> 4, S = d.RS & 15); tr == -3: zero d.K doubles at address d.src (the BN
  //             statistics slabs); tr == -4: add 1 to d.K int64 counters at address d.src
  //             (num_batches_tracked)
  if (d.tr == -2) {
    const int R = d.RS >> 4, S = d.RS & 15;
    const long long n = (long long)d.K * 256;
    for (long long i = (long long)blockIdx.x * 256 + tid; i < n; i += (long long)gridDim.x * 256) {
      const int k = (int)(i >> 8), r = (int)(i >> 5) & 7, s = (int)(i >> 2) & 7, c = (int)i & 3;
      const bool v = r < R && s < S && c < d.C;
      wbuf[d.fwd + i] = v ? (bf16)master[d.src + (((long long)k * R + r) * S + s) * d.C + c] : (bf16)0.f;
    }
    return;
  }
  if (d.tr == -3) {
    double* z = reinterpret_cast<double*>(d.src);
    const long long n2 = (long long)d.K / 2;
    for (long long i = (long long)blockIdx.x * 256 + tid; i < n2; i += (long long)gridDim.x * 256)
      reinterpret_cast<f64x2*>(z)[i] = f64x2{0.0, 0.0};
    if ((d.K & 1) && blockIdx.x == 0 && tid == 0) z[d.K - 1] = 0.0;
    return;
  }
  if (d.tr == -4) {
    long long* c = reinterpret_cast<long long*>(d.src);
    if (blockIdx.x == 0)
      for (int i = tid; i < d.K; i += 256) c[i] += 1;
    return;
  }
  if (d.tr < 0) {
    const long long n = (long long)d.K * d.RS * d.C;
    const long long n4 = n / 4;
    for (long long i = (long long)blockIdx.x * 256 + tid; i < n4; i += (long long)gridDim.x * 256)
      *reinterpret_cast<bf16x4*>(wbuf + d.fwd + 4 * i) = load4_bf16(master + d.src + 4 * i);
    for (long long i = 4 * n4 + (long long)blockIdx.x * 256 + tid; i < n; i += (long long)gridDim.x * 256)
      wbuf[d.fwd + i] = (bf16)master[d.src + i];
    return;
  }
  __shared__ bf16 tile[64][64 + 4];
  const int tk = d.K / 64, tc = d.C / 64, ntiles = tk * tc * d.RS;
  const int rs = d.RS * d.C;  // master row length (per k)
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int kc = t / d.RS, tap = t - kc * d.RS;
    const int k0 = (kc / tc) * 64, c0 = (kc - (kc / tc) * tc) * 64;
    // load 64 k-rows x 64 channels (fp32, 4 per thread per pass), write the KRSC bf16 copy
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int kr = p * 16 + (tid >> 4), cq = (tid & 15) * 4;
      const long long e = (long long)(k0 + kr) * rs + tap * d.C + c0 + cq;
      const bf16x4 b = load4_bf16(master + d.src + e);
      *reinterpret_cast<bf16x4*>(wbuf + d.fwd + e) = b;
      tile[kr][cq] = b[0]; tile[kr][cq + 1] = b[1]; tile[kr][cq + 2] = b[2]; tile[kr][cq + 3] = b[3];
    }
    __syncthreads();
    // transposed CRSK: row (c, tap), 64 consecutive k
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int cr = p * 16 + (tid >> 4), kq = (tid & 15) * 4;
      const bf16x4 b = {tile[kq][cr], tile[kq + 1][cr], tile[kq + 2][cr], tile[kq + 3][cr]};
      *reinterpret_cast<bf16x4*>(wbuf + d.tr + ((long long)(c0 + cr) * d.RS + tap) * d.K + k0 + kq) = b;
    }
    __syncthreads();
  }
}

__global__ void cast_f32_bf16_kernel(const float* __restrict__ x, bf16* __restrict__ y, long long n) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) y[i] = (bf16)x[i];
}
__global__ void cast_bf16_f32_kernel(const bf16* __restrict__ x, float* __restrict__ y, long long n, float scale, int accumulate) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    y[i] = (accumulate ? y[i] : 0.f) + scale * (float)x[i];
}

}  // namespace dbx

// ======================================================================================
// C ABI launchers
// ======================================================================================
using namespace dbx;

// grid cap of an elementwise pass whose every block also finalizes all C channels of a BN
static inline int fin_cap(int C) {
  const int c = (512 * 256) / (C > 0 ? C : 1);
  return c < 512 ? 512 : (c > 4096 ? 4096 : c);
}
static inline int grid_for(long long n, int block = 256, int cap = 8192) {
  long long g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}
#define RET_LAST return (int)hipGetLastError()

extern "C" int dbx_bn_finalize(const double* stats, int nshard, int C, float count, const float* gamma,
                               const float* beta, float eps, float momentum, float* rm, float* rv,
                               float* scale, float* shift, float* save_mean, float* save_invstd, hipStream_t st) {
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 7) / 8), dim3(256), 0, st, stats, nshard, C, count, gamma,
                     beta, eps, momentum, rm, rv, scale, shift, save_mean, save_invstd);
  RET_LAST;
}
extern "C" int dbx_bn_eval_coeff(int C, const float* gamma, const float* beta, float eps, const float* rm,
                                 const float* rv, float* scale, float* shift, hipStream_t st) {
  hipLaunchKernelGGL(bn_eval_coeff_kernel, dim3((C + 255) / 256), dim3(256), 0, st, C, gamma, beta, eps, rm, rv, scale, shift);
  RET_LAST;
}
extern "C" int dbx_channel_stats(const bf16* y, long long M, int C, double* stats, int nshard, hipStream_t st) {
  if (C % 8 || C / 8 > 256) return -1;
  const int rpb = 256 / (C / 8);
  hipLaunchKernelGGL(channel_stats_kernel, dim3(grid_for(M, rpb, 2048)), dim3(256), 0, st, y, M, C, stats, nshard);
  RET_LAST;
}
extern "C" int dbx_bn_apply(const bf16* y, const float* sc, const float* sh, const bf16* res, const float* rsc,
                            const float* rsh, bf16* out, long long n, int C, int res_mode, int relu,
                            unsigned char* mbits, hipStream_t st, const BnFin* fin, const BnFin* rfin) {
  if (n % C || C % 8 || C / 8 > 256) return -1;
  if (rfin && res_mode != 2) return -2;
  const long long M = n / C;
  // (with an in-launch finalize every block derives all C channels' affine: fewer, fatter blocks)
  const dim3 g(grid_for(M, 256 / (C / 8), (fin || rfin) ? fin_cap(C) : 4096)), b(256);
#define BA(R, A) hipLaunchKernelGGL((bn_apply_kernel<R, A>), g, b, 0, st, y, sc, sh, res, rsc, rsh, out, mbits, M, C, fin, rfin)
  if (res_mode == 0) { if (relu) BA(0, true); else BA(0, false); }
  else if (res_mode == 1) { if (relu) BA(1, true); else BA(1, false); }
  else { if (relu) BA(2, true); else BA(2, false); }
#undef BA
  RET_LAST;
}
extern "C" int dbx_bn_bwd_reduce(const bf16* dout, const bf16* mref, const bf16* y, const float* sc, const float* sh,
                                 const float* mean, const float* invstd, long long M, int C, double* stats,
                                 int nshard, int mask_mode, hipStream_t st) {
  if (C % 8 || C / 8 > 256) return -1;
  const int rpb = 256 / (C / 8);
  const dim3 g(grid_for(M, rpb, 2048)), b(256);
  if (mask_mode == 0) hipLaunchKernelGGL((bn_bwd_reduce_kernel<0>), g, b, 0, st, dout, mref, y, sc, sh, mean, invstd, M, C, stats, nshard);
  else if (mask_mode == 1) hipLaunchKernelGGL((bn_bwd_reduce_kernel<1>), g, b, 0, st, dout, mref, y, sc, sh, mean, invstd, M, C, stats, nshard);
  else hipLaunchKernelGGL((bn_bwd_reduce_kernel<2>), g, b, 0, st, dout, mref, y, sc, sh, mean, invstd, M, C, stats, nshard);
  RET_LAST;
}
extern "C" int dbx_bn_bwd_coeff(const double* stats, int nshard, int C, float count, const float* gamma,
                                const float* mean, const float* invstd, float* coeff, float* dgamma, float* dbeta,
                                int accumulate, hipStream_t st) {
  hipLaunchKernelGGL(bn_bwd_coeff_kernel, dim3((C + 7) / 8), dim3(256), 0, st, stats, nshard, C, count, gamma,
                     mean, invstd, coeff, dgamma, dbeta, accumulate);
  RET_LAST;
}
extern "C" int dbx_bn_bwd_apply(const bf16* dout, const bf16* mref, const bf16* y, const float* sc, const float* sh,
                                const float* coeff, bf16* dy, bf16* gout, long long n, int C, int mask_mode,
                                hipStream_t st, const BnFin* fin) {
  if (n % C || C % 8 || C / 8 > 256) return -1;
  const long long M = n / C;
  // (with the in-launch finalize every block derives all C coefficients: fewer, fatter blocks --
  // as many as keep that work per launch about C x 512 channel-finalizes)
  const dim3 g(grid_for(M, 256 / (C / 8), fin ? fin_cap(C) : 4096)), b(256);
#define BB(MK, WG) hipLaunchKernelGGL((bn_bwd_apply_kernel<MK, WG>), g, b, 0, st, dout, mref, y, sc, sh, coeff, dy, gout, M, C, fin)
  if (mask_mode == 0) { if (gout) BB(0, true); else BB(0, false); }
  else if (mask_mode == 1) { if (gout) BB(1, true); else BB(1, false); }
  else { if (gout) BB(2, true); else BB(2, false); }
#undef BB
  RET_LAST;
}
extern "C" int dbx_bn_bwd_apply2(const bf16* g, const bf16* y1, const float* c1, bf16* dy1, const bf16* y2,
                                 const float* c2, bf16* dy2, long long n, int C, hipStream_t st, const BnFin* fin1,
                                 const BnFin* fin2) {
  if (n % C || C % 8 || C / 8 > 256) return -1;
  const long long M = n / C;
  hipLaunchKernelGGL(bn_bwd_apply2_kernel, dim3(grid_for(M, 256 / (C / 8), (fin1 || fin2) ? fin_cap(C) : 4096)), dim3(256), 0, st, g, y1, c1, dy1,
                     y2, c2, dy2, M, C, fin1, fin2);
  RET_LAST;
}
extern "C" int dbx_maxpool_fwd(const bf16* x, const float* sc, const float* sh, bf16* out, unsigned char* arg,
                               bf16* ymax, int N, int H, int W, int C, int P, int Q, int K, int stride, int pad, int relu,
                               hipStream_t st, const BnFin* fin) {
  if (C % 8) return -1;
  if (C / 8 > 256) return -1;
  if (fin && !sc) return -2;
  const dim3 grid(grid_for((long long)N * P * Q, 256 / (C / 8), fin ? 1024 : 4096));
  if (K == 3 && (long long)N * P * Q < (1ll << 31))
    hipLaunchKernelGGL(maxpool_fwd_kernel<3>, grid, dim3(256), 0, st, x, sc, sh, out, arg, ymax, N, H, W, C, P, Q, K,
                       stride, pad, relu, fin);
  else
    hipLaunchKernelGGL(maxpool_fwd_kernel<0>, grid, dim3(256), 0, st, x, sc, sh, out, arg, ymax, N, H, W, C, P, Q, K,
                       stride, pad, relu, fin);
  RET_LAST;
}
extern "C" int dbx_maxpool_bwd(const bf16* dout, const unsigned char* arg, bf16* dx, int N, int H, int W, int C, int P,
                               int Q, int K, int stride, int pad, hipStream_t st) {
  if (C % 8) return -1;
  const long long total = (long long)N * H * W * (C / 8);
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(grid_for(total)), dim3(256), 0, st, dout, arg, dx, N, H, W, C, P, Q, K,
                     stride, pad);
  RET_LAST;
}
extern "C" int dbx_pool_bn_bwd(const bf16* dpool, const unsigned char* arg, const bf16* y, const float* sc,
                               const float* sh, const float* c1, const float* c2, const float* c3, bf16* dy,
                               double* stats, int nshard, int N, int H, int W, int C, int P, int Q, int K, int stride,
                               int pad, int apply, hipStream_t st) {
  if (C % 8 || 256 % (C / 8) || (K + stride - 1) / stride > 2) return -1;
  if ((long long)N * H * W * C >= (1LL << 31) || (long long)N * P * Q * C >= (1LL << 31)) return -2;
  const dim3 g(grid_for((long long)N * H, 1, apply ? 8192 : 2048)), b(256);
  if (apply)
    hipLaunchKernelGGL((pool_bn_bwd_kernel<true>), g, b, 0, st, dpool, arg, y, sc, sh, c1, c2, c3, dy, stats, nshard,
                       N, H, W, C, P, Q, K, stride, pad);
  else
    hipLaunchKernelGGL((pool_bn_bwd_kernel<false>), g, b, 0, st, dpool, arg, y, sc, sh, c1, c2, c3, dy, stats, nshard,
                       N, H, W, C, P, Q, K, stride, pad);
  RET_LAST;
}
extern "C" int dbx_avgpool_fwd(const bf16* x, bf16* out, int N, int HW, int C, hipStream_t st) {
  if (C % 8) return -1;
  hipLaunchKernelGGL(avgpool_fwd_kernel, dim3((C / 8 + 63) / 64, N), dim3(64), 0, st, x, out, N, HW, C);
  RET_LAST;
}
extern "C" int dbx_avgpool_bwd(const bf16* dout, bf16* dx, int N, int HW, int C, hipStream_t st) {
  if (C % 8) return -1;
  hipLaunchKernelGGL(avgpool_bwd_kernel, dim3(grid_for((long long)N * HW * C / 8)), dim3(256), 0, st, dout, dx, N, HW, C);
  RET_LAST;
}
extern "C" int dbx_softmax_ce(const void* logits, int is_bf16, const long long* labels, void* dlogits, float* loss_out,
                              double* stats, int B, int C, float smoothing, float gscale, const long long* labels2,
                              const float* lam, hipStream_t st) {
  if (is_bf16)
    hipLaunchKernelGGL(softmax_ce_kernel<bf16>, dim3(B), dim3(256), 0, st, (const bf16*)logits, labels, (bf16*)dlogits,
                       loss_out, stats, B, C, smoothing, gscale, labels2, lam);
  else
    hipLaunchKernelGGL(softmax_ce_kernel<float>, dim3(B), dim3(256), 0, st, (const float*)logits, labels,
                       (float*)dlogits, loss_out, stats, B, C, smoothing, gscale, labels2, lam);
  RET_LAST;
}
extern "C" int dbx_sgd(float* p, const float* g, float* v, bf16* p16, long long n, const float* hyper, float lr,
                       float mom, float damp, float wd, int nesterov, int first, const float* gscale_ptr, float gscale,
                       hipStream_t st) {
  hipLaunchKernelGGL(sgd_kernel, dim3(grid_for((n + 3) / 4)), dim3(256), 0, st, p, g, v, p16, n, hyper, lr, mom, damp,
                     wd, nesterov, first, gscale_ptr, gscale);
  RET_LAST;
}
extern "C" int dbx_adam(float* p, const float* g, float* m, float* v, bf16* p16, long long n, const float* hyper,
                        float lr, float b1, float b2, float eps, float wd, int decoupled, float bc1, float bc2,
                        const float* gscale_ptr, float gscale, hipStream_t st) {
  hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n)), dim3(256), 0, st, p, g, m, v, p16, n, hyper, lr, b1, b2, eps, wd,
                     decoupled, bc1, bc2, gscale_ptr, gscale);
  RET_LAST;
}
extern "C" int dbx_lars_scale(const float* p, float* g, const int* seg_off, const int* seg_len, const int* adapt,
                              int nseg, int max_len, double* norms, float gs, float eta, float wd, hipStream_t st) {
  if (nseg <= 0) return 0;
  int bx = (int)((max_len + 255) / 256);
  bx = bx < 1 ? 1 : (bx > kLarsMaxBlocks ? kLarsMaxBlocks : bx);
  hipLaunchKernelGGL(lars_norms_kernel, dim3(bx, nseg), dim3(256), 0, st, p, g, seg_off, seg_len, gs, norms);
  hipLaunchKernelGGL(lars_apply_kernel, dim3(bx, nseg), dim3(256), 0, st, p, g, seg_off, seg_len, adapt, norms, gs,
                     eta, wd);
  RET_LAST;
}
extern "C" int dbx_sumsq(const float* x, long long n, double* out, hipStream_t st) {
  hipLaunchKernelGGL(sumsq_kernel, dim3(grid_for(n, 256, 1024)), dim3(256), 0, st, x, n, out);
  RET_LAST;
}
extern "C" int dbx_clip_factor(const double* sumsq, float max_norm, float* out, hipStream_t st) {
  hipLaunchKernelGGL(clip_factor_kernel, dim3(1), dim3(1), 0, st, sumsq, max_norm, out);
  RET_LAST;
}
extern "C" int dbx_normalize_u8(const unsigned char* in, bf16* out, const unsigned char* flip, int N, int H, int W,
                                int Cin, float m0, float m1, float m2, float s0, float s1, float s2, hipStream_t st) {
  hipLaunchKernelGGL(normalize_u8_kernel, dim3(grid_for((long long)N * H * W)), dim3(256), 0, st, in, out, flip, N, H, W,
                     Cin, m0, m1, m2, s0, s1, s2);
  RET_LAST;
}
extern "C" int dbx_augment_u8(const unsigned char* in, bf16* out, const float* boxes, const unsigned char* flip, int N,
                              int Hin, int Win, int Cin, int Ho, int Wo, float m0, float m1, float m2, float s0, float s1,
                              float s2, const int* perm, const int* mixbox, hipStream_t st) {
  hipLaunchKernelGGL(augment_u8_kernel, dim3(N * Ho < 4096 ? N * Ho : 4096), dim3(Wo >= 256 ? 256 : ((Wo + 63) / 64) * 64), 0, st, in, out, boxes, flip, N,
                     Hin, Win, Cin, Ho, Wo, m0, m1, m2, s0, s1, s2, perm, mixbox);
  RET_LAST;
}
extern "C" int dbx_weight_prep(const float* master, bf16* wbuf, const void* desc_dev, int nlayers, hipStream_t st) {
  hipLaunchKernelGGL(weight_prep_kernel<float>, dim3(512, nlayers), dim3(256), 0, st, master, wbuf,
                     (const WDesc*)desc_dev, nlayers);
  RET_LAST;
}
extern "C" int dbx_weight_prep16(const bf16* src, bf16* wbuf, const void* desc_dev, int nlayers, hipStream_t st) {
  hipLaunchKernelGGL(weight_prep_kernel<bf16>, dim3(512, nlayers), dim3(256), 0, st, src, wbuf,
                     (const WDesc*)desc_dev, nlayers);
  RET_LAST;
}
extern "C" int dbx_cast_f32_bf16(const float* x, bf16* y, long long n, hipStream_t st) {
  hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3(grid_for(n)), dim3(256), 0, st, x, y, n);
  RET_LAST;
}
extern "C" int dbx_cast_bf16_f32(const bf16* x, float* y, long long n, float scale, int accumulate, hipStream_t st) {
  hipLaunchKernelGGL(cast_bf16_f32_kernel, dim3(grid_for(n)), dim3(256), 0, st, x, y, n, scale, accumulate);
  RET_LAST;
}
