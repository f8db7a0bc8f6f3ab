// Shared helpers for the CDNA4 (gfx950) kernels of dbx_distributed_pytorch_examples_amd.
// Wave = 64 lanes; MFMA = v_mfma_f32_16x16x32_bf16; all activations NHWC bf16.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define DBX_LDS __attribute__((address_space(3)))

#define HIP_CHECK_RET(expr)                                   \
  do {                                                        \
    hipError_t _e = (expr);                                   \
    if (_e != hipSuccess) return (int)_e;                     \
  } while (0)

__device__ __forceinline__ float bf2f(bf16 v) { return (float)v; }
__device__ __forceinline__ bf16 f2bf(float v) { return (bf16)v; }

// 16-byte vector of 8 bf16 <-> 8 floats
__device__ __forceinline__ void unpack8(const u32x4 v, float* f) {
  const bf16x8 b = __builtin_bit_cast(bf16x8, v);
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = (float)b[j];
}
__device__ __forceinline__ u32x4 pack8(const float* f) {
  bf16x8 b;
#pragma unroll
  for (int j = 0; j < 8; ++j) b[j] = (bf16)f[j];
  return __builtin_bit_cast(u32x4, b);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Bijective XCD-aware remap of a linear workgroup id (cdna_hip_programming.md §5 "XCD swizzle
// must be bijective"): blocks b and b+8 share an XCD, so give each XCD group a contiguous range
// of logical tiles; tiles adjacent in logical order then share that XCD's L2.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7;
  const int q = nwg >> 3, r = nwg & 7;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

static inline int cdiv(int a, int b) { return (a + b - 1) / b; }
