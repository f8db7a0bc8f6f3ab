// HBM roof probe for gfx950: hand-written streaming kernels with dwordx4 loads / stores, the
// read:write mixes of the framework's HBM-bound convolutions, plain vs non-temporal accesses, and
// one pass whose working set fits the last-level cache (MALL). Replaces the stock-PyTorch "roof"
// of tools/hbm_roof.py (whose copy / sum kernels are not tuned to this part).
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/bin/hbm_probe tools/hbm_probe.hip
//   tools/bin/hbm_probe [GiB per stream = 1] [iters = 10]
//
// Each line: mix (reads:writes streams), access kind, grid shape, bytes moved, time, TB/s.
// The TAIL data gradient at 56x56 reads dy, the BN-backward operand and the pre-BN tensor and
// writes dx, the applied gradient and the shortcut gradient, with the mask / stats on top: a
// 5:2 mix is the closest pure-stream analogue; 2:1 is the prologue / epilogue conv mix.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                        \
    }                                                                                      \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ f4 ld(const f4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NT>
__device__ __forceinline__ void st(f4* p, f4 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// R input streams, W output streams, n f4 elements each; UNROLL independent f4 per lane per trip
// so several loads are in flight before the first use. W == 0: a per-block partial sum is written
// (so the reads are not dead code).
template <int R, int W, bool NT, int UNROLL>
__global__ __launch_bounds__(256) void stream_kernel(const f4* const* __restrict__ in, f4* const* __restrict__ out,
                                                      long long n, float* __restrict__ sink) {
  const long long stride = (long long)gridDim.x * blockDim.x * UNROLL;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  for (long long base = (long long)blockIdx.x * blockDim.x * UNROLL + threadIdx.x; base < n; base += stride) {
    f4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) v[u] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < R; ++r) {
      f4 t[UNROLL];
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        long long i = base + (long long)u * blockDim.x;
        t[u] = i < n ? ld<NT>(in[r] + i) : f4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) v[u] += t[u];
    }
    if constexpr (W == 0) {
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) acc += v[u];
    } else {
#pragma unroll
      for (int w = 0; w < W; ++w)
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
          long long i = base + (long long)u * blockDim.x;
          if (i < n) st<NT>(out[w] + i, v[u] * (float)(w + 1));
        }
    }
  }
  if constexpr (W == 0) {
    float s = acc.x + acc.y + acc.z + acc.w;
    if (s == 1234.5f) sink[blockIdx.x] = s;  // practically never true; keeps the loads live
  }
}

struct Bufs {
  std::vector<f4*> p;
  f4** d_in = nullptr;
  f4** d_out = nullptr;
};

template <int R, int W, bool NT, int UNROLL>
double run(const Bufs& b, long long n, int grid, int iters, float* sink) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto launch = [&] {
    hipLaunchKernelGGL((stream_kernel<R, W, NT, UNROLL>), dim3(grid), dim3(256), 0, 0, (const f4* const*)b.d_in,
                       b.d_out, n, sink);
  };
  for (int i = 0; i < 2; ++i) launch();
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  for (int i = 0; i < iters; ++i) launch();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return ms / iters;
}

template <int R, int W, bool NT, int UNROLL>
void row(const char* name, const Bufs& b, long long n, int grid, int iters, float* sink) {
  double ms = run<R, W, NT, UNROLL>(b, n, grid, iters, sink);
  double bytes = (double)(R + (W ? W : 0)) * n * 16.0;
  std::printf("%-6s %-4s unroll %d grid %7d  %8.3f GiB  %8.3f ms  %6.2f TB/s\n", name, NT ? "nt" : "std", UNROLL,
              grid, bytes / (1 << 30), ms, bytes / (ms * 1e-3) / 1e12);
  std::fflush(stdout);
}

template <int R, int W>
void sweep(const char* name, const Bufs& b, long long n, int iters, float* sink, int cus) {
  // persistent grids (k workgroups per CU) and one full grid (one trip per lane)
  for (int k : {4, 8, 16}) {
    row<R, W, false, 4>(name, b, n, cus * k, iters, sink);
    row<R, W, true, 4>(name, b, n, cus * k, iters, sink);
  }
  int full = (int)((n + 256LL * 2 - 1) / (256LL * 2));
  row<R, W, false, 2>(name, b, n, full, iters, sink);
  row<R, W, true, 2>(name, b, n, full, iters, sink);
}

int main(int argc, char** argv) {
  double gib = argc > 1 ? std::atof(argv[1]) : 1.0;
  int iters = argc > 2 ? std::atoi(argv[2]) : 10;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  std::printf("# %s  %d CUs  L2 %d KiB per XCD  memory clock %d kHz bus %d bit\n", prop.gcnArchName, cus,
              prop.l2CacheSize / 1024, prop.memoryClockRate, prop.memoryBusWidth);
  const int kStreams = 7;
  auto alloc = [&](long long n) {
    Bufs b;
    for (int i = 0; i < kStreams; ++i) {
      f4* p;
      CK(hipMalloc(&p, n * sizeof(f4)));
      CK(hipMemset(p, 0, n * sizeof(f4)));
      b.p.push_back(p);
    }
    // inputs: streams 0..4, outputs: streams 5, 6 (the 1:1 copy reads 0 and writes 5)
    std::vector<f4*> in(b.p.begin(), b.p.begin() + 5), out(b.p.begin() + 5, b.p.end());
    CK(hipMalloc(&b.d_in, 5 * sizeof(f4*)));
    CK(hipMalloc(&b.d_out, 2 * sizeof(f4*)));
    CK(hipMemcpy(b.d_in, in.data(), 5 * sizeof(f4*), hipMemcpyHostToDevice));
    CK(hipMemcpy(b.d_out, out.data(), 2 * sizeof(f4*), hipMemcpyHostToDevice));
    return b;
  };
  auto release = [&](Bufs& b) {
    for (auto p : b.p) CK(hipFree(p));
    CK(hipFree(b.d_in));
    CK(hipFree(b.d_out));
  };
  float* sink;
  CK(hipMalloc(&sink, 1 << 20));

  const long long n = (long long)(gib * (1LL << 30)) / 16;
  std::printf("# HBM: %.2f GiB per stream (7 streams allocated, %.1f GiB)\n", gib, 7 * gib);
  {
    Bufs b = alloc(n);
    sweep<1, 0>("read", b, n, iters, sink, cus);
    sweep<0, 1>("write", b, n, iters, sink, cus);
    sweep<1, 1>("1:1", b, n, iters, sink, cus);
    sweep<2, 1>("2:1", b, n, iters, sink, cus);
    sweep<5, 2>("5:2", b, n, iters, sink, cus);
    release(b);
  }
  // last-level-cache-sized working set: 1:1 over 2 x 64 MiB, 5:2 over 7 x 16 MiB
  {
    const long long m = (64LL << 20) / 16;
    Bufs b = alloc(m);
    std::printf("# LLC-sized: 1:1 over 2 x 64 MiB\n");
    row<1, 1, false, 4>("1:1", b, m, cus * 8, iters * 10, sink);
    row<1, 1, true, 4>("1:1", b, m, cus * 8, iters * 10, sink);
    release(b);
    const long long m2 = (16LL << 20) / 16;
    Bufs b2 = alloc(m2);
    std::printf("# LLC-sized: 5:2 over 7 x 16 MiB\n");
    row<5, 2, false, 4>("5:2", b2, m2, cus * 8, iters * 10, sink);
    row<5, 2, true, 4>("5:2", b2, m2, cus * 8, iters * 10, sink);
    release(b2);
  }
  CK(hipFree(sink));
  return 0;
}
