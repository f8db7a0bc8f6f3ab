// The reference's MNIST ``Net`` (`01_torch_distributor/01_basic_torch_distributor.py:75-91`, the one
// path of the reference that really trains data-parallel) as two fused HIP kernels, fp32 end to end:
//
//   conv5x5(1->10) -> maxpool2 -> relu -> conv5x5(10->20) -> Dropout2d -> maxpool2 -> relu
//   -> fc 320->50 -> relu -> dropout -> fc 50->10 -> log_softmax
//
// The whole network is 21,840 parameters and ~0.5 MFLOP per image forward: on the stock stack every
// op is its own tiny launch (~20 forward + ~30 backward kernels per step, each far from filling a
// GPU). Here ONE workgroup carries one image through the whole forward with every activation in
// LDS, and one through the whole backward (input-gradient chain + the weight gradients of that
// image), writing the image's gradient contribution to its own slab; a reduce kernel sums the slabs
// in image order (deterministic, no atomics). Dropout / Dropout2d masks come from counter-based
// Philox draws (seed, offset, element), so the backward regenerates the forward's masks.
//
// Parameter layout (flat, module registration order): conv1.w [10][1][5][5], conv1.b [10],
// conv2.w [20][10][5][5], conv2.b [20], fc1.w [50][320], fc1.b [50], fc2.w [10][50], fc2.b [10].
#include "common.h"

namespace dbx {
namespace mnist {

constexpr int OFF_C1W = 0, OFF_C1B = 250, OFF_C2W = 260, OFF_C2B = 5260, OFF_F1W = 5280, OFF_F1B = 21280;
constexpr int OFF_F2W = 21330, OFF_F2B = 21830, NPARAM = 21840;

__device__ __forceinline__ unsigned philox(unsigned long long idx, unsigned long long seed, unsigned offset) {
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
// keep-scale (0 or 1/(1-p)) of element idx of a dropout stream; p = 0.5 in the reference
__device__ __forceinline__ float keep(unsigned long long idx, unsigned long long seed, unsigned offset, int train) {
  if (!train) return 1.f;
  return philox(idx, seed, offset) < 0x80000000u ? 2.f : 0.f;
}

struct Saved {           // per image, written by the forward for the backward
  float a1[1440];        // relu(maxpool(conv1)) [10][12][12]
  float a2[320];         // relu(maxpool(dropout2d(conv2))) [20][4][4] (the fc1 input, flatten order)
  float h1[50];          // relu(fc1) before dropout
  float logp[10];
  unsigned char i1[1440];  // argmax in the 2x2 window of pool 1 (dy*2 + dx)
  unsigned char i2[320];
};

}  // namespace mnist

using namespace mnist;

// one workgroup (256 threads) per image
__global__ __launch_bounds__(256) void mnist_fwd_kernel(const float* __restrict__ x, const float* __restrict__ P,
                                                        Saved* __restrict__ sv, float* __restrict__ logp_out,
                                                        unsigned long long seed, unsigned offset, int train) {
  __shared__ float sx[784], sc1[5760], sa1[1440], sc2[1280], sa2[320], sh1[50], sz[16];
  const int n = blockIdx.x, t = threadIdx.x;
  for (int i = t; i < 784; i += 256) sx[i] = x[(size_t)n * 784 + i];
  __syncthreads();
  // conv1 5x5, 1 -> 10, 28 -> 24
  for (int o = t; o < 5760; o += 256) {
    const int c = o / 576, r = o - c * 576, y = r / 24, xx = r - y * 24;
    float s = P[OFF_C1B + c];
    const float* w = P + OFF_C1W + c * 25;
#pragma unroll
    for (int i = 0; i < 5; ++i)
#pragma unroll
      for (int j = 0; j < 5; ++j) s += w[i * 5 + j] * sx[(y + i) * 28 + xx + j];
    sc1[o] = s;
  }
  __syncthreads();
  // maxpool 2 (first max wins ties, as torch) + relu -> a1 [10][12][12]
  for (int o = t; o < 1440; o += 256) {
    const int c = o / 144, r = o - c * 144, y = r / 12, xx = r - y * 12;
    const float* b = sc1 + c * 576 + (2 * y) * 24 + 2 * xx;
    float m = b[0];
    int k = 0;
    if (b[1] > m) { m = b[1]; k = 1; }
    if (b[24] > m) { m = b[24]; k = 2; }
    if (b[25] > m) { m = b[25]; k = 3; }
    sa1[o] = fmaxf(m, 0.f);
    sv[n].i1[o] = (unsigned char)k;
    sv[n].a1[o] = fmaxf(m, 0.f);
  }
  __syncthreads();
  // conv2 5x5, 10 -> 20, 12 -> 8; Dropout2d (per image and channel)
  for (int o = t; o < 1280; o += 256) {
    const int c = o / 64, r = o - c * 64, y = r / 8, xx = r - y * 8;
    float s = P[OFF_C2B + c];
    const float* w = P + OFF_C2W + c * 250;
    for (int k = 0; k < 10; ++k) {
      const float* a = sa1 + k * 144 + y * 12 + xx;
#pragma unroll
      for (int i = 0; i < 5; ++i)
#pragma unroll
        for (int j = 0; j < 5; ++j) s += w[k * 25 + i * 5 + j] * a[i * 12 + j];
    }
    sc2[o] = s * keep((unsigned long long)n * 20 + c, seed, offset, train);
  }
  __syncthreads();
  // maxpool 2 + relu -> a2 [20][4][4]
  for (int o = t; o < 320; o += 256) {
    const int c = o / 16, r = o - c * 16, y = r / 4, xx = r - y * 4;
    const float* b = sc2 + c * 64 + (2 * y) * 8 + 2 * xx;
    float m = b[0];
    int k = 0;
    if (b[1] > m) { m = b[1]; k = 1; }
    if (b[8] > m) { m = b[8]; k = 2; }
    if (b[9] > m) { m = b[9]; k = 3; }
    sa2[o] = fmaxf(m, 0.f);
    sv[n].i2[o] = (unsigned char)k;
    sv[n].a2[o] = fmaxf(m, 0.f);
  }
  __syncthreads();
  // fc1 320 -> 50 + relu: 4 lanes per output (partial dot products + shuffle)
  if (t < 200) {
    const int h = t >> 2, q = t & 3;
    const float* w = P + OFF_F1W + h * 320;
    float s = 0.f;
    for (int k = q; k < 320; k += 4) s += w[k] * sa2[k];
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    if (q == 0) {
      const float v = fmaxf(s + P[OFF_F1B + h], 0.f);
      sh1[h] = v;
      sv[n].h1[h] = v;
    }
  }
  __syncthreads();
  // dropout + fc2 50 -> 10 + log_softmax
  if (t < 64) {
    float z = -INFINITY;
    if (t < 10) {
      z = P[OFF_F2B + t];
      for (int h = 0; h < 50; ++h) z += P[OFF_F2W + t * 50 + h] * sh1[h] * keep((unsigned long long)n * 50 + h, seed, offset + 1, train);
    }
    const float m = wave_max(z);
    const float e = t < 10 ? __expf(z - m) : 0.f;
    const float lse = m + __logf(wave_sum(e));
    if (t < 10) {
      sv[n].logp[t] = z - lse;
      logp_out[(size_t)n * 10 + t] = z - lse;
    }
  }
}

// one workgroup per image: the image's gradient contribution -> its slab gws[n][NPARAM]
__global__ __launch_bounds__(256) void mnist_bwd_kernel(const float* __restrict__ x, const float* __restrict__ P,
                                                        const Saved* __restrict__ sv, const float* __restrict__ dlogp,
                                                        float* __restrict__ gws, unsigned long long seed,
                                                        unsigned offset) {
  __shared__ float sx[784], sa1[1440], sa2[320], sh1d[50], sdz[16], sdh1[50], sda2[320], sdc2[1280], sdc1[5760];
  __shared__ float sred[16];
  const int n = blockIdx.x, t = threadIdx.x;
  float* g = gws + (size_t)n * NPARAM;
  const Saved& S = sv[n];
  for (int i = t; i < 784; i += 256) sx[i] = x[(size_t)n * 784 + i];
  for (int i = t; i < 1440; i += 256) sa1[i] = S.a1[i];
  for (int i = t; i < 320; i += 256) sa2[i] = S.a2[i];
  if (t < 50) sh1d[t] = S.h1[t] * keep((unsigned long long)n * 50 + t, seed, offset + 1, 1);
  // log_softmax backward: dz = g - softmax * sum(g)
  if (t < 64) {
    const float gg = t < 10 ? dlogp[(size_t)n * 10 + t] : 0.f;
    const float sg = wave_sum(gg);
    if (t < 10) sdz[t] = gg - __expf(S.logp[t]) * sg;
  }
  __syncthreads();
  // fc2: dW = dz h1d^T, db = dz; dh1d = W^T dz -> dropout -> relu'
  for (int i = t; i < 500; i += 256) g[OFF_F2W + i] = sdz[i / 50] * sh1d[i % 50];
  if (t < 10) g[OFF_F2B + t] = sdz[t];
  if (t < 50) {
    float s = 0.f;
    for (int j = 0; j < 10; ++j) s += P[OFF_F2W + j * 50 + t] * sdz[j];
    s *= keep((unsigned long long)n * 50 + t, seed, offset + 1, 1);
    sdh1[t] = S.h1[t] > 0.f ? s : 0.f;
  }
  __syncthreads();
  // fc1: dW = dh1 a2^T, db = dh1; da2 = W^T dh1
  for (int i = t; i < 16000; i += 256) g[OFF_F1W + i] = sdh1[i / 320] * sa2[i % 320];
  if (t < 50) g[OFF_F1B + t] = sdh1[t];
  for (int k = t; k < 320; k += 256) {
    float s = 0.f;
    for (int h = 0; h < 50; ++h) s += P[OFF_F1W + h * 320 + k] * sdh1[h];
    sda2[k] = s;
  }
  for (int i = t; i < 1280; i += 256) sdc2[i] = 0.f;
  __syncthreads();
  // relu' + maxpool-2 backward (argmax routing) + Dropout2d -> d conv2 output
  for (int o = t; o < 320; o += 256) {
    const int c = o / 16, r = o - c * 16, y = r / 4, xx = r - y * 4;
    const float d = sa2[o] > 0.f ? sda2[o] : 0.f;
    const int k = S.i2[o];
    sdc2[c * 64 + (2 * y + (k >> 1)) * 8 + 2 * xx + (k & 1)] = d * keep((unsigned long long)n * 20 + c, seed, offset, 1);
  }
  __syncthreads();
  // conv2 weight / bias gradients: dW[c][k][i][j] = sum_{y,x} dc2[c][y][x] a1[k][y+i][x+j]
  for (int wi = t; wi < 5000; wi += 256) {
    const int c = wi / 250, r = wi - c * 250, k = r / 25, ij = r - k * 25, i = ij / 5, j = ij - i * 5;
    const float* d = sdc2 + c * 64;
    const float* a = sa1 + k * 144 + i * 12 + j;
    float s = 0.f;
#pragma unroll 8
    for (int p = 0; p < 64; ++p) s += d[p] * a[(p >> 3) * 12 + (p & 7)];
    g[OFF_C2W + wi] = s;
  }
  if (t < 20) {
    float s = 0.f;
    for (int p = 0; p < 64; ++p) s += sdc2[t * 64 + p];
    g[OFF_C2B + t] = s;
  }
  // d a1 = full correlation of dc2 with the flipped conv2 weights, then relu' and pool-1 routing
  for (int i = t; i < 5760; i += 256) sdc1[i] = 0.f;
  __syncthreads();
  for (int o = t; o < 1440; o += 256) {
    const int k = o / 144, r = o - k * 144, yy = r / 12, xx = r - yy * 12;
    float s = 0.f;
    for (int c = 0; c < 20; ++c) {
      const float* w = P + OFF_C2W + c * 250 + k * 25;
      const float* d = sdc2 + c * 64;
#pragma unroll
      for (int i = 0; i < 5; ++i) {
        const int y = yy - i;
        if (y < 0 || y >= 8) continue;
#pragma unroll
        for (int j = 0; j < 5; ++j) {
          const int xq = xx - j;
          if (xq >= 0 && xq < 8) s += w[i * 5 + j] * d[y * 8 + xq];
        }
      }
    }
    const float dv = sa1[o] > 0.f ? s : 0.f;
    const int kk = S.i1[o];
    sdc1[k * 576 + (2 * yy + (kk >> 1)) * 24 + 2 * xx + (kk & 1)] = dv;
  }
  __syncthreads();
  // conv1 weight / bias gradients
  for (int wi = t; wi < 250; wi += 256) {
    const int c = wi / 25, ij = wi - c * 25, i = ij / 5, j = ij - i * 5;
    const float* d = sdc1 + c * 576;
    float s = 0.f;
    for (int p = 0; p < 576; ++p) s += d[p] * sx[(p / 24 + i) * 28 + p % 24 + j];
    g[OFF_C1W + wi] = s;
  }
  if (t < 10) {
    float s = 0.f;
    for (int p = 0; p < 576; ++p) s += sdc1[t * 576 + p];
    g[OFF_C1B + t] = s;
  }
}

// grad[p] = sum over images of gws[n][p], in image order (deterministic)
__global__ void mnist_reduce_kernel(const float* __restrict__ gws, float* __restrict__ grad, int N) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= NPARAM) return;
  float s = 0.f;
  for (int n = 0; n < N; ++n) s += gws[(size_t)n * NPARAM + p];
  grad[p] = s;
}

}  // namespace dbx

using namespace dbx;

extern "C" long long dbx_mnist_saved_bytes() { return (long long)sizeof(mnist::Saved); }

extern "C" int dbx_mnist_fwd(const float* x, const float* params, void* saved, float* logp, int N,
                             unsigned long long seed, unsigned offset, int train, hipStream_t st) {
  if (N <= 0) return -70;
  hipLaunchKernelGGL(mnist_fwd_kernel, dim3(N), dim3(256), 0, st, x, params, (mnist::Saved*)saved, logp, seed, offset,
                     train);
  return (int)hipGetLastError();
}

extern "C" int dbx_mnist_bwd(const float* x, const float* params, const void* saved, const float* dlogp, float* gws,
                             float* grad, int N, unsigned long long seed, unsigned offset, hipStream_t st) {
  if (N <= 0) return -70;
  hipLaunchKernelGGL(mnist_bwd_kernel, dim3(N), dim3(256), 0, st, x, params, (const mnist::Saved*)saved, dlogp, gws,
                     seed, offset);
  hipLaunchKernelGGL(mnist_reduce_kernel, dim3((mnist::NPARAM + 255) / 256), dim3(256), 0, st, gws, grad, N);
  return (int)hipGetLastError();
}
