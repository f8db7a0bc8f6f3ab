// BatchNorm finalize math shared by the standalone kernels (nn_ops.hip bn_finalize_kernel /
// bn_bwd_coeff_kernel) and the in-launch finalize of the conv epilogue (bn_fin_tail): one
// definition, so a fused and an unfused step produce the same bits.
#pragma once
#include "abi.h"
#include "common.h"

namespace dbx {

// forward: shard sums (s, q) of channel c -> the affine (scale, shift) and the batch moments
__device__ __forceinline__ void bn_fwd_affine(int c, double s, double q, float count, const float* gamma,
                                              const float* beta, float eps, float& scale, float& shift,
                                              double& mean, double& var, float& invstd) {
#pragma clang fp contract(off)  // no context-dependent FMA contraction: fused == standalone bits
  mean = s / count;
  var = q / count - mean * mean;
  if (var < 0.0) var = 0.0;
  invstd = (float)(1.0 / sqrt(var + (double)eps));
  const float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
  scale = g * invstd;
  shift = b - (float)mean * g * invstd;
}

// forward: shard sums (s, q) of channel c -> scale / shift, saved mean / invstd, running stats
__device__ __forceinline__ void bn_fwd_final(int c, double s, double q, float count, const float* gamma,
                                             const float* beta, float eps, float momentum, float* running_mean,
                                             float* running_var, float* scale, float* shift, float* save_mean,
                                             float* save_invstd) {
#pragma clang fp contract(off)
  double mean, var;
  float invstd, sc, sh;
  bn_fwd_affine(c, s, q, count, gamma, beta, eps, sc, sh, mean, var, invstd);
  scale[c] = sc;
  shift[c] = sh;
  if (save_mean) save_mean[c] = (float)mean;
  if (save_invstd) save_invstd[c] = invstd;
  if (running_mean && momentum > 0.f) {
    const double unbiased = count > 1.f ? var * count / (count - 1.0) : var;
    running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * (float)mean;
    running_var[c] = (1.f - momentum) * running_var[c] + momentum * (float)unbiased;
  }
}

// backward: shard sums (sum g, sum g*xhat) of channel c -> dy = k1*g + k2*y + k3, dgamma, dbeta
__device__ __forceinline__ void bn_bwd_k(double sd, double qd, float count, float g, float is, float mu, float& k1,
                                         float& k2, float& k3) {
#pragma clang fp contract(off)
  const float s = (float)sd, q = (float)qd;
  const float sg = s / count, sgx = q / count;
  k1 = g * is;
  k2 = -g * is * is * sgx;
  k3 = -g * is * sg + g * is * is * sgx * mu;
}
__device__ __forceinline__ void bn_bwd_final(int C, int c, double sd, double qd, float count, const float* gamma,
                                             const float* mean, const float* invstd, float* coeff, float* dgamma,
                                             float* dbeta, int accumulate) {
#pragma clang fp contract(off)
  const float s = (float)sd, q = (float)qd;
  float k1, k2, k3;
  bn_bwd_k(sd, qd, count, gamma ? gamma[c] : 1.f, invstd[c], mean[c], k1, k2, k3);
  coeff[c] = k1; coeff[C + c] = k2; coeff[2 * C + c] = k3;
  if (dgamma) dgamma[c] = (accumulate ? dgamma[c] : 0.f) + q;
  if (dbeta) dbeta[c] = (accumulate ? dbeta[c] : 0.f) + s;
}

// Shard sum of channel c in the standalone kernels' order (0 + shard 0 + shard 1 + ...: their
// 32-way split holds one shard per lane for nshard <= 32, summed lane by lane). The in-launch
// finalize reads the shards with agent-scope (sc1) loads: they bypass this CU's L1, and the shards'
// lines are never in an L2 (the statistics atomics execute at the memory side and drop the line).
// The loads are issued 16 shards at a time before their in-order adds: one memory round trip per 16
// shards instead of one per shard (the shards live at the memory side, ~1-2 us away).
__device__ __forceinline__ void bn_fin_sums_sc1(const double* stats, int nshard, int C, int c, double& s, double& q) {
  s = 0.0;
  q = 0.0;
  for (int k0 = 0; k0 < nshard; k0 += 16) {
    double sv[16], qv[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int k = k0 + j < nshard ? k0 + j : k0;  // (past the end: a valid address, not added)
      gf64* p = (gf64*)(stats + (size_t)k * 2 * C + c);
      sv[j] = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      qv[j] = __hip_atomic_load(p + C, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      if (k0 + j < nshard) {
        s += sv[j];
        q += qv[j];
      }
    }
  }
}

__device__ __forceinline__ void bn_fin_channel(const BnFin& f, int c) {
  double s, q;
  bn_fin_sums_sc1(f.stats, f.nshard, f.C, c, s, q);
  if (f.mode == 1)
    bn_fwd_final(c, s, q, f.count, f.gamma, f.beta, f.eps, f.momentum, f.running_mean, f.running_var, f.scale,
                 f.shift, f.mean, f.invstd);
  else
    bn_bwd_final(f.C, c, s, q, f.count, f.gamma, f.mean, f.invstd, f.coeff, f.dgamma, f.dbeta, f.accumulate);
}

// Consumer-side forward finalize (IGemmArgs::fin_in): the prologue affine of channel c, summed over
// the shards in the standalone kernels' order (plain loads: the statistics were completed by an
// earlier launch); the storing workgroup also writes every bn_finalize output of the channel.
__device__ __forceinline__ void bn_fin_consume(const BnFin& f, int c, bool store, float& scale, float& shift) {
  double s = 0.0, q = 0.0;
  for (int k0 = 0; k0 < f.nshard; k0 += 16) {  // loads batched ahead of the in-order adds
    double sv[16], qv[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int k = k0 + j < f.nshard ? k0 + j : k0;
      sv[j] = f.stats[(size_t)k * 2 * f.C + c];
      qv[j] = f.stats[(size_t)k * 2 * f.C + f.C + c];
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      if (k0 + j < f.nshard) {
        s += sv[j];
        q += qv[j];
      }
    }
  }
  if (store) {
    bn_fwd_final(c, s, q, f.count, f.gamma, f.beta, f.eps, f.momentum, f.running_mean, f.running_var, f.scale,
                 f.shift, f.mean, f.invstd);
    scale = f.scale[c];
    shift = f.shift[c];
    return;
  }
  double mean, var;
  float invstd;
  bn_fwd_affine(c, s, q, f.count, f.gamma, f.beta, f.eps, scale, shift, mean, var, invstd);
}

// End of a conv tile epilogue whose launch carries BN finalize descriptors: once every wave's
// statistics atomics have completed (they execute at the memory side: no L2 write-back, so no
// release fence -- a buffer_wbl2 per tile would write back the tile's just-stored outputs, which
// measured 1.6x slower steps), one lane per 64-channel group takes a ticket; the tile that completes
// a group's count (all ceil(M / BM) M-tiles of the producer, over all its launches) finalizes those
// 64 channels from sc1 loads of the shards (/opt/skills/guides/MI355X_MICROARCH.md, the image's CDNA4 guide, "Valid forms", row 1: the last
// adder loads after its add returned, the other waves after a barrier), then resets the counter.
// The finalizing block reads 2 x nshard x 64 doubles. n0: first output channel of the tile.
template <int BM, int BN>
__device__ __forceinline__ void bn_fin_tail(const IGemmArgs& a, const int n0, bf16* lds) {
  constexpr int G = BN / 64;
  static_assert(G >= 1 && G * 64 == BN, "64-channel groups");
  const int tid = threadIdx.x;
  const int ng = a.fin2 ? 2 * G : G;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's statistics atomics have completed
  __syncthreads();                                   // ... every wave's; the LDS is free
  int* flag = reinterpret_cast<int*>(lds);
  if (tid < ng) {
    const BnFin* f = tid < G ? a.fin1 : a.fin2;
    const unsigned total = a.fin_final ? (unsigned)(a.fin_base + (a.M + BM - 1) / BM) : 0xFFFFFFFFu;
    const unsigned t = __hip_atomic_fetch_add((gu32*)(f->cnt + (n0 >> 6) + tid % G), 1u, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
    flag[tid] = t + 1u == total;
  }
  __syncthreads();
  for (int k = 0; k < ng; ++k) {
    if (!flag[k]) continue;  // block-uniform
    const BnFin* f = k < G ? a.fin1 : a.fin2;
    const int g = (n0 >> 6) + k % G;
    if (tid < 64) bn_fin_channel(*f, g * 64 + tid);
    if (tid == 0) __hip_atomic_store((gu32*)(f->cnt + g), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();  // flags read before the LDS is reused
}

}  // namespace dbx
