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
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef double f64x2 __attribute__((ext_vector_type(2)));
// global-address-space views for inter-workgroup counters and sc1 loads (global_, never flat_ ops)
typedef __attribute__((address_space(1))) unsigned gu32;
typedef __attribute__((address_space(1))) double gf64;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define DBX_LDS __attribute__((address_space(3)))

// Device-side index checks of the debug build (build_ext with DBX_DEBUG=1 -> _C_variant_debug):
// a failing condition prints itself with the block / thread; the kernel continues (no trap, so a
// failing check cannot take the device down). Compiled out of the production build.
#ifdef DBX_DEBUG
#define DBX_DCHECK(cond)                                                                              \
  do {                                                                                                \
    if (!(cond))                                                                                      \
      printf("[dbx] DBX_DCHECK failed: %s at %s:%d block %d thread %d\n", #cond, __FILE__, __LINE__, \
             (int)blockIdx.x, (int)threadIdx.x);                                                      \
  } while (0)
#else
#define DBX_DCHECK(cond) \
  do {                   \
  } while (0)
#endif

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
__device__ __forceinline__ unsigned pack2(float lo, float hi) {
  typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
  const bf16x2_t b = {(__bf16)lo, (__bf16)hi};
  return __builtin_bit_cast(unsigned, b);
}
__device__ __forceinline__ u32x4 pack8(const float* f) {
  bf16x8 b;
#pragma unroll
  for (int j = 0; j < 8; ++j) b[j] = (bf16)f[j];
  return __builtin_bit_cast(u32x4, b);
}

// ReLU of 8 packed bf16: a bf16 bit pattern read as int16 is negative exactly when the value is
// (incl. -0), so max(x, 0) is one v_pk_max_i16 per 2 elements instead of 2 fp32 max
typedef short s16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ u32x4 relu_bf16x8(const u32x4 v) {
  const s16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
  return __builtin_bit_cast(u32x4, __builtin_elementwise_max(__builtin_bit_cast(s16x8, v), z));
}

// floor(x / d) for 0 <= x, x * d < 2^40 with mag = ceil(2^40 / d) (host: div_magic)
__device__ __forceinline__ int mdiv(int x, unsigned long long mag) {
  return (int)(((unsigned long long)(unsigned)x * mag) >> 40);
}
// x / d via the magic when the host provided one (uniform branch), else a plain division
__device__ __forceinline__ int mdiv_or(int x, unsigned long long mag, int d) {
  return mag ? mdiv(x, mag) : x / d;
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

// Raw buffer loads (SRD in SGPRs, 32-bit per-lane byte offset). An offset at or past num_records
// returns zeros, which is how the conv gathers zero-fill padding taps and rows past M without a
// select on the data; built from kernel arguments only, so the descriptor is provably uniform.
typedef __amdgpu_buffer_rsrc_t rsrc_t;
constexpr unsigned kOOB = 0xFFFFFF00u;  // an offset no tensor reaches (num_records <= kOOB)
__device__ __forceinline__ rsrc_t make_rsrc(const void* p, unsigned long long bytes) {
  const unsigned n = bytes < (unsigned long long)kOOB ? (unsigned)bytes : kOOB;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)n, 0x00020000);
}
__device__ __forceinline__ u32x4 buf_load16(rsrc_t r, unsigned off) {
  return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
__device__ __forceinline__ void buf_store8(rsrc_t r, unsigned off, unsigned char v) {
  __builtin_amdgcn_raw_buffer_store_b8(v, r, off, 0, 0);
}
// a store at an out-of-range offset is dropped by the hardware (branch-free conditional store)
__device__ __forceinline__ void buf_store16(rsrc_t r, unsigned off, u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v), r, off, 0, 0);
}

// ---- LDS-DMA (gfx950 buffer_load_dwordx4 ... lds) ----------------------------------------------
// 16 bytes per lane go from a raw buffer straight into LDS at m0 + 16*lane: 1 KiB per
// wave-instruction, no VGPR staging and no ds_write (the LDS write path of a register-staged
// tile costs ~13 cycles per ds_write_b128 and was the largest LDS consumer of the conv loops).
// Out-of-range offsets land zeros, like buf_load16. Issued through inline asm: hipcc's waitcnt
// pass treats its own LDS-DMA builtin as an LDS store of unknown address and inserts vmcnt(0)
// before every later ds_read, which would drain the prefetch pipeline; the caller instead waits
// with dma_wait<N>() (counted vmcnt) + a barrier before it reads a filled buffer. The asm is
// invisible to that pass, so its own vmcnt waits count fewer loads than are in flight: they
// only ever over-wait, never under-wait.
typedef int i32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ i32x4 make_srd(const void* p, unsigned long long bytes) {
  const unsigned long long a = (unsigned long long)p;
  const unsigned n = bytes < (unsigned long long)kOOB ? (unsigned)bytes : kOOB;
  return i32x4{(int)(unsigned)a, (int)((unsigned)(a >> 32) & 0xFFFFu), (int)n, 0x00020000};
}
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void lds_dma16(const i32x4 srd, unsigned voff, unsigned lds_byte) {
  // m0 = the wave's 1 KiB destination (wave-uniform by construction; readfirstlane makes it SGPR)
  const unsigned m = __builtin_amdgcn_readfirstlane(lds_byte);
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(m), "v"(voff), "s"(srd)
               : "memory", "m0");
}
#pragma clang diagnostic pop
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(unsigned long long)(const DBX_LDS void*)p;
}
// wait until at most N vector-memory operations of this wave are outstanding (loads, stores and
// LDS-DMA count together, in issue order); expcnt / lgkmcnt left unconstrained
template <int N>
__device__ __forceinline__ void dma_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

// XOR swizzle of a [rows][nch x 16B] LDS tile image read by ds_read_b64_tr_b16 (weight gradients):
__device__ __forceinline__ int tr_swz(int row, int ch, int nch) {
  // conflict-free for BOTH the ds_write_b128 staging stores (8-lane groups: the two rows a group
  // covers must land on different 64-B halves of the 128-B bank window) and the
  // ds_read_b64_tr_b16 fragment reads (32-lane groups over 8 rows); model: tools/lds_banks.py
  if (nch == 32) return ch ^ (((row & 1) << 1) | ((row & 2) << 1) | (row & 8));  // 256-wide tiles
  if (nch == 16) return ch ^ ((((row & 1) << 2) | (row & 2) | (row & 8)) & 15);
  return ch ^ ((((row & 1) << 2) ^ (row & 2) ^ (((row >> 3) & 1) << 2)) & 7);
}

