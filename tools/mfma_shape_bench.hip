// v_mfma_f32_16x16x32_bf16 vs v_mfma_f32_32x32x16_bf16 in the eight-wave conv kernel's inner loop
// ("add a 32x32x16 main loop ... or keep the A/B showing why it loses").
//
// Both variants run the fast_igemm_kernel geometry (csrc/conv_fast.hip): a 256 x 256 x 64 operand
// stage resident in LDS (XOR-swizzled rows of 128 B), 8 waves per workgroup (2 per SIMD), one
// workgroup per CU, a 128 x 64 output tile per wave (128 fp32 accumulators per lane either way),
// fragments read with ds_read_b128 and fed to the MFMAs; random bf16 operands (the clock the chip
// holds depends on the data: MI355X_MICROARCH.md 'DVFS give-back'). Per 64-deep stage a wave reads
// 24 fragments (16 x 16 x 32: 2 k-steps x (8 A + 4 B); 32 x 32 x 16: 4 k-steps x (4 A + 2 B)) and
// issues 64 resp. 32 MFMAs -- the same LDS bytes and the same MFMA cycles (16 vs 32 per
// instruction), so the A/B isolates the instruction shape. Optional: one __syncthreads per stage
// (the ring barrier of the real kernel).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/mfma_shape_bench tools/mfma_shape_bench.hip
//   tools/bin/mfma_shape_bench [stages=4096] [grid=256] [rounds=3]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));     \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

constexpr int BM = 256, BN = 256, BK = 64, WM = 2, WN = 4;
__device__ __forceinline__ int swz(int row) { return (row >> 1) & 7; }

// fill the LDS stage from global (once), then loop over `stages` re-reading it
template <int SHAPE, bool BAR>
__global__ __launch_bounds__(512, 1) void mfma_loop(const bf16* __restrict__ src, float* __restrict__ out, int stages) {
  __shared__ __attribute__((aligned(16))) bf16 lds[(BM + BN) * BK];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wm = wid / WN, wn = wid % WN;
  for (int i = tid; i < (BM + BN) * BK / 8; i += 512) {
    const int row = i / 8, ch = i % 8;
    *reinterpret_cast<bf16x8*>(lds + row * BK + ((ch ^ swz(row)) << 3)) =
        *reinterpret_cast<const bf16x8*>(src + ((size_t)blockIdx.x * 64 + (size_t)i * 8) % (1 << 20));
  }
  __syncthreads();
  const bf16* sA = lds;
  const bf16* sB = lds + BM * BK;
  if constexpr (SHAPE == 16) {
    constexpr int TM = BM / (16 * WM), TN = BN / (16 * WN);  // 8 x 4
    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int st = 0; st < stages; ++st) {
#pragma unroll
      for (int ks = 0; ks < BK / 32; ++ks) {
        bf16x8 af[TM], bfr[TN];
        const int ch = ks * 4 + (lane >> 4);
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int row = wn * (BN / WN) + j * 16 + (lane & 15);
          bfr[j] = *reinterpret_cast<const bf16x8*>(sB + row * BK + ((ch ^ swz(row)) << 3));
        }
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int row = wm * (BM / WM) + i * 16 + (lane & 15);
          af[i] = *reinterpret_cast<const bf16x8*>(sA + row * BK + ((ch ^ swz(row)) << 3));
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
      }
      if (BAR) __syncthreads();
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) s += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    out[blockIdx.x * 512 + tid] = s;
  } else {
    // 32 x 32 x 16: lane l holds row (l % 32), k = 8 * (l / 32) .. +7 of a 32 x 16 operand
    constexpr int TM = BM / (32 * WM), TN = BN / (32 * WN);  // 4 x 2
    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    for (int st = 0; st < stages; ++st) {
#pragma unroll
      for (int ks = 0; ks < BK / 16; ++ks) {
        bf16x8 af[TM], bfr[TN];
        const int ch = ks * 2 + (lane >> 5);  // 16-B chunk of the 128-B row
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int row = wn * (BN / WN) + j * 32 + (lane & 31);
          bfr[j] = *reinterpret_cast<const bf16x8*>(sB + row * BK + ((ch ^ swz(row)) << 3));
        }
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int row = wm * (BM / WM) + i * 32 + (lane & 31);
          af[i] = *reinterpret_cast<const bf16x8*>(sA + row * BK + ((ch ^ swz(row)) << 3));
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
      }
      if (BAR) __syncthreads();
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) s += acc[i][j][r];
    out[blockIdx.x * 512 + tid] = s;
  }
}

template <int SHAPE, bool BAR>
static double run(const bf16* src, float* out, int stages, int grid, int reps) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL((mfma_loop<SHAPE, BAR>), dim3(grid), dim3(512), 0, 0, src, out, stages);  // warm-up
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((mfma_loop<SHAPE, BAR>), dim3(grid), dim3(512), 0, 0, src, out, stages);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0.f;
  CHECK(hipEventElapsedTime(&ms, a, b));
  const double flop = 2.0 * BM * BN * BK * (double)stages * grid * reps;
  return flop / (ms * 1e-3) / 1e12;
}

int main(int argc, char** argv) {
  const int stages = argc > 1 ? atoi(argv[1]) : 4096;
  const int grid = argc > 2 ? atoi(argv[2]) : 256;
  const int rounds = argc > 3 ? atoi(argv[3]) : 3;
  const size_t n = (1 << 20) + 4096;
  std::vector<uint16_t> h(n);
  uint32_t x = 12345;
  for (size_t i = 0; i < n; ++i) {  // random bf16 in about [-2, 2]
    x = x * 1664525u + 1013904223u;
    const float f = ((x >> 8) & 0xFFFF) / 16384.0f - 2.0f;
    uint32_t u;
    std::memcpy(&u, &f, 4);
    h[i] = (uint16_t)(u >> 16);
  }
  bf16* src;
  float* out;
  CHECK(hipMalloc(&src, n * 2));
  CHECK(hipMalloc(&out, (size_t)grid * 512 * 4));
  CHECK(hipMemcpy(src, h.data(), n * 2, hipMemcpyHostToDevice));
  printf("# 256x256x64 stage in LDS, 8 waves (2/SIMD), 128x64 per wave, random bf16, %d stages x %d WGs\n", stages, grid);
  for (int r = 0; r < rounds; ++r) {  // interleaved rounds: clock drift hits both shapes alike
    const double a0 = run<16, false>(src, out, stages, grid, 5);
    const double b0 = run<32, false>(src, out, stages, grid, 5);
    const double a1 = run<16, true>(src, out, stages, grid, 5);
    const double b1 = run<32, true>(src, out, stages, grid, 5);
    printf("round %d: 16x16x32 %.0f TF/s | 32x32x16 %.0f TF/s (ratio %.3f) ; with a barrier per stage: 16x16x32 %.0f | 32x32x16 %.0f (ratio %.3f)\n",
           r, a0, b0, b0 / a0, a1, b1, b1 / a1);
  }
  return 0;
}
