// Direct two-shot all-reduce over peer-mapped buffers: the xGMI-aware path for small / medium
// gradient buckets (the reference only reaches NCCL through c10d,
// 01_torch_distributor/01_basic_torch_distributor.py:269, and sets NCCL_DEBUG in
// setup/00_setup.py:122-123).
//
// An MI355X node is a full xGMI mesh: every GPU has a direct link to each of its 7 peers. A ring
// all-reduce crosses 2(n-1) = 14 dependent steps and drives two links per ring; the two-shot form
// below reaches every peer directly in two steps:
//   reduce-scatter: rank r sums segment r of every rank's buffer (reads 1/n of the buffer from each
//                   peer, all seven links at once) and writes the sum into its own segment r;
//   all-gather:     rank r copies segment j from rank j for every j != r.
// Bytes per link per rank are 2S/n either way (S = the buffer), so the direct form has the ring's
// bandwidth term at a fraction of its latency term: the win is on the buffers that are latency
// bound (parallel/collective_plan.py prices both).
//
// Synchronisation is per workgroup: workgroup b of every rank owns the same stripe of every
// segment, so only the b-th workgroups of the ranks meet, at three flag barriers (entry: every
// rank's producers are done; middle: every rank's reduce-scatter reads of my buffer are done; exit:
// every rank's all-gather reads of my buffer are done, so the stream may overwrite it next). A
// barrier: every wave drains its stores, one lane releases at system scope (writes the XCD's L2
// back), lanes 0..n-1 store the generation into rank j's flag slot (uncached memory), then poll
// their own slots and acquire at system scope before any peer data is read. Generations live in
// device memory (one counter per workgroup), so a launch captured into a HIP graph replays
// correctly. Every poll is bounded by a wall-clock deadline (s_memrealtime, 100 MHz): a missing
// peer ends the wait with an error bit instead of a wave that never finishes. A workgroup whose
// barrier timed out skips the rest of the protocol (no further waits) and writes NaN over every
// element it owns in the result, so a partial sum can never pass as a gradient; the error bit also
// lands in a pinned host word that the comm watchdog polls without a device sync.
#include "common.h"

namespace dbx {

constexpr int DAR_MAX_RANKS = 8;
constexpr int DAR_THREADS = 256;

struct DarArgs {
  float* buf[DAR_MAX_RANKS];        // this call's range in every rank's buffer (rank order)
  unsigned* flags[DAR_MAX_RANKS];   // every rank's flag array: [3 phases][grid][DAR_MAX_RANKS] (uncached)
  unsigned* gen;                    // this rank's per-workgroup generation counters [grid]
  int* err;                         // this rank's error word (bit 0: a barrier timed out)
  int* err_host;                    // device view of a pinned host word mirroring err (may be null)
  long long n;                      // elements
  long long seg;                    // elements per segment (multiple of 4)
  unsigned long long timeout_ticks; // per barrier, in s_memrealtime ticks (100 MHz)
  int rank, world;
};

__device__ __forceinline__ unsigned* dar_slot(unsigned* f, int phase, int b, int grid, int src) {
  return f + ((size_t)phase * grid + b) * DAR_MAX_RANKS + src;
}

// the kernel body of rank `rank`'s workgroup b of G (rank / gen / err given apart from the shared args)
__device__ __forceinline__ void dar_body(const DarArgs& a, const int rank, unsigned* const gen, int* const err,
                                         int* const err_host, const int b, const int G) {
  const int tid = threadIdx.x;
  __shared__ unsigned s_gen;
  __shared__ int s_bad;
  if (tid == 0) {
    s_gen = gen[b] + 1u;
    s_bad = 0;
  }
  __syncthreads();
  const unsigned g = s_gen;

  auto barrier = [&](int phase) __attribute__((always_inline)) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave: its stores have completed
    __syncthreads();
    if (tid < 64) {  // wave 0 signals and waits for the workgroup
      if (tid == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: L2 written back
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (tid < a.world)
        __hip_atomic_store(dar_slot(a.flags[tid], phase, b, G, rank), g, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
      if (tid < a.world) {
        unsigned* f = dar_slot(a.flags[rank], phase, b, G, tid);
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        // generations only grow; (int)(v - g) < 0 is "not yet" across a 2^32 wrap too
        while ((int)(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - g) < 0) {
          if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout_ticks) {
            s_bad = 1;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      if (tid == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: no stale peer lines
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
  };

  const long long n = a.n, S = a.seg;
  auto seg_lo = [&](int r) __attribute__((always_inline)) { const long long lo = (long long)r * S; return lo < n ? lo : n; };
  auto seg_hi = [&](int r) __attribute__((always_inline)) { const long long hi = (long long)(r + 1) * S; return hi < n ? hi : n; };
  const long long stride = (long long)G * DAR_THREADS;

  // a timed-out barrier: poison every element this workgroup owns in the result (its stripe of every
  // segment) and leave without waiting again
  auto poison = [&]() __attribute__((always_inline)) {
    const float qnan = __builtin_nanf("");
    for (int j = 0; j < a.world; ++j) {
      const long long lo = seg_lo(j), hi = seg_hi(j);
      for (long long i = lo + (long long)b * DAR_THREADS + tid; i < hi; i += stride) a.buf[rank][i] = qnan;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      gen[b] = g;
      atomicOr(err, 1);
      if (err_host) __hip_atomic_store(err_host, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  };

  barrier(0);  // entry: every rank's producers of this range have finished
  if (s_bad) {
    poison();
    return;
  }
  {
    // reduce-scatter: my segment, summed over ranks in rank order (the same order on every rank:
    // each segment is reduced by exactly one rank, so all ranks end with identical bits)
    const long long lo = seg_lo(rank), hi = seg_hi(rank);
    const long long n4 = (hi - lo) >> 2;
    for (long long i = (long long)b * DAR_THREADS + tid; i < n4; i += stride) {
      f32x4 v[DAR_MAX_RANKS];
#pragma unroll
      for (int j = 0; j < DAR_MAX_RANKS; ++j)  // every peer's load in flight before the first add
        if (j < a.world) v[j] = *reinterpret_cast<const f32x4*>(a.buf[j] + lo + 4 * i);
      f32x4 s = v[0];
#pragma unroll
      for (int j = 1; j < DAR_MAX_RANKS; ++j)
        if (j < a.world) s += v[j];
      *reinterpret_cast<f32x4*>(a.buf[rank] + lo + 4 * i) = s;
    }
    // scalar tail (only the last segment can end off a 4-element boundary)
    const long long t = lo + 4 * n4 + (long long)b * DAR_THREADS + tid;
    if (b * DAR_THREADS + tid < 4 && t < hi) {
      float s = a.buf[0][t];
      for (int j = 1; j < a.world; ++j) s += a.buf[j][t];
      a.buf[rank][t] = s;
    }
  }
  barrier(1);  // every rank's reduce-scatter reads of my buffer are done; every reduced segment is published
  if (s_bad) {
    poison();
    return;
  }
  for (int jj = 1; jj < a.world; ++jj) {
    // all-gather: segment j from rank j (start at my right neighbour: the ranks spread their reads)
    const int j = (rank + jj) % a.world;
    const long long lo = seg_lo(j), hi = seg_hi(j);
    const long long n4 = (hi - lo) >> 2;
    for (long long i = (long long)b * DAR_THREADS + tid; i < n4; i += stride)
      *reinterpret_cast<f32x4*>(a.buf[rank] + lo + 4 * i) = *reinterpret_cast<const f32x4*>(a.buf[j] + lo + 4 * i);
    const long long t = lo + 4 * n4 + (long long)b * DAR_THREADS + tid;
    if (b * DAR_THREADS + tid < 4 && t < hi) a.buf[rank][t] = a.buf[j][t];
  }
  barrier(2);  // exit: every rank's all-gather reads of my buffer are done
  if (tid == 0) {
    gen[b] = g;
    // the data is complete here; a late peer only delays its own exit, but the bit still ends the job
    if (s_bad) {
      atomicOr(err, 1);
      if (err_host) __hip_atomic_store(err_host, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

__global__ __launch_bounds__(DAR_THREADS) void dar_kernel(const DarArgs a) {
  dar_body(a, a.rank, a.gen, a.err, a.err_host, blockIdx.x, gridDim.x);
}

// Test form: every rank of one process in ONE dispatch (workgroup = rank * G + b), so the ranks are
// co-resident by construction -- the protocol checked on one GPU without depending on how streams
// map to hardware queues (two "ranks" on one queue would serialise and time out).
struct DarMultiArgs {
  DarArgs base;                      // buf / flags / n / seg / timeout / world (rank, gen, err unused)
  unsigned* gen[DAR_MAX_RANKS];
  int* err[DAR_MAX_RANKS];
  int grid;
};

__global__ __launch_bounds__(DAR_THREADS) void dar_multi_kernel(const DarMultiArgs m) {
  const int r = blockIdx.x / m.grid, b = blockIdx.x - r * m.grid;
  dar_body(m.base, r, m.gen[r], m.err[r], nullptr, b, m.grid);
}

}  // namespace dbx

using namespace dbx;

// peers / flags: world device pointers each (rank order). Returns a hipError_t code, or -70.. for
// argument errors (checked again on the Python side).
extern "C" int dbx_dar_launch(float* const* bufs, unsigned* const* flags, unsigned* gen, int* err, int* err_host,
                              long long n, int rank, int world, int grid, double timeout_s, hipStream_t st) {
  if (world < 1 || world > DAR_MAX_RANKS || rank < 0 || rank >= world) return -70;
  if (grid < 1 || n < 0) return -71;
  DarArgs a{};
  for (int j = 0; j < world; ++j) {
    if (!bufs[j] || !flags[j] || (reinterpret_cast<uintptr_t>(bufs[j]) & 15)) return -72;
    a.buf[j] = bufs[j];
    a.flags[j] = flags[j];
  }
  a.gen = gen;
  a.err = err;
  a.err_host = err_host;
  a.n = n;
  a.seg = ((n + world - 1) / world + 3) & ~3LL;
  a.timeout_ticks = (unsigned long long)(timeout_s * 1e8);
  a.rank = rank;
  a.world = world;
  hipLaunchKernelGGL(dar_kernel, dim3(grid), dim3(DAR_THREADS), 0, st, a);
  return (int)hipGetLastError();
}

// flags of one rank: 3 phases x grid x DAR_MAX_RANKS words in uncached device memory (peer stores
// land in memory, local polls read memory), zeroed; gen / err in ordinary device memory, zeroed;
// err_host: a zeroed pinned host word, mapped for the device (its device address in *err_host_dev)
extern "C" int dbx_dar_alloc(int grid, void** flags, void** gen, void** err, void** err_host, void** err_host_dev) {
  const size_t fb = sizeof(unsigned) * 3 * (size_t)grid * DAR_MAX_RANKS;
  HIP_CHECK_RET(hipExtMallocWithFlags(flags, fb, hipDeviceMallocUncached));
  HIP_CHECK_RET(hipMemset(*flags, 0, fb));
  HIP_CHECK_RET(hipMalloc(gen, sizeof(unsigned) * grid));
  HIP_CHECK_RET(hipMemset(*gen, 0, sizeof(unsigned) * grid));
  HIP_CHECK_RET(hipMalloc(err, sizeof(int)));
  HIP_CHECK_RET(hipMemset(*err, 0, sizeof(int)));
  HIP_CHECK_RET(hipHostMalloc(err_host, sizeof(int), hipHostMallocMapped | hipHostMallocCoherent));
  *reinterpret_cast<volatile int*>(*err_host) = 0;
  HIP_CHECK_RET(hipHostGetDevicePointer(err_host_dev, *err_host, 0));
  return (int)hipDeviceSynchronize();
}

extern "C" int dbx_dar_free(void* flags, void* gen, void* err, void* err_host) {
  if (flags) (void)hipFree(flags);
  if (gen) (void)hipFree(gen);
  if (err) (void)hipFree(err);
  if (err_host) (void)hipHostFree(err_host);
  return 0;
}

extern "C" int dbx_dar_max_ranks() { return DAR_MAX_RANKS; }

extern "C" int dbx_dar_launch_multi(float* const* bufs, unsigned* const* flags, unsigned* const* gens,
                                    int* const* errs, long long n, int world, int grid, double timeout_s,
                                    hipStream_t st) {
  if (world < 1 || world > DAR_MAX_RANKS || grid < 1 || n < 0) return -70;
  DarMultiArgs m{};
  for (int j = 0; j < world; ++j) {
    if (!bufs[j] || !flags[j] || (reinterpret_cast<uintptr_t>(bufs[j]) & 15)) return -72;
    m.base.buf[j] = bufs[j];
    m.base.flags[j] = flags[j];
    m.gen[j] = gens[j];
    m.err[j] = errs[j];
  }
  m.base.n = n;
  m.base.seg = ((n + world - 1) / world + 3) & ~3LL;
  m.base.timeout_ticks = (unsigned long long)(timeout_s * 1e8);
  m.base.world = world;
  m.grid = grid;
  hipLaunchKernelGGL(dar_multi_kernel, dim3(grid * world), dim3(DAR_THREADS), 0, st, m);
  return (int)hipGetLastError();
}
