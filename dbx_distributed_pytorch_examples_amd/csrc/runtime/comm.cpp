// Native collective layer: an RCCL communicator owned by the framework.
//
// The reference reaches NCCL only through c10d (`dist.init_process_group("nccl")`,
// 01_torch_distributor/01_basic_torch_distributor.py:269) and DDP's reducer. Here the engine can
// drive RCCL itself: one communicator per process group, collectives enqueued on the caller's HIP
// stream (the trainer's comm stream), no c10d work objects, no watchdog thread -- so the bucket
// collectives can be recorded into the same HIP graph as the backward segments that produce
// them (RCCL launches are ordinary stream work under capture).
//
// RCCL is resolved at run time from the librccl the process already has (torch's own, so there is
// exactly one RCCL instance and one set of xGMI channels per process), falling back to
// /opt/rocm/lib. Nothing links against it at build time: the extension still loads on hosts
// without RCCL, and every entry point then raises.
#include <chrono>
#include <dlfcn.h>
#include <unistd.h>
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include <pybind11/stl.h>

extern "C" {
int dbx_dar_launch(float* const*, unsigned* const*, unsigned*, int*, int*, long long, int, int, int, double, hipStream_t);
int dbx_dar_alloc(int, void**, void**, void**, void**, void**);
int dbx_dar_free(void*, void*, void*, void*);
int dbx_dar_max_ranks();
int dbx_dar_launch_multi(float* const*, unsigned* const*, unsigned* const*, int* const*, long long, int, int, double,
                         hipStream_t);
}

namespace py = pybind11;

namespace dbx {
namespace comm {

struct Api {
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*comm_init_rank_config)(ncclComm_t*, int, ncclUniqueId, int, ncclConfig_t*) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*comm_abort)(ncclComm_t) = nullptr;
  ncclResult_t (*comm_count)(const ncclComm_t, int*) = nullptr;
  ncclResult_t (*comm_get_async_error)(ncclComm_t, ncclResult_t*) = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*reduce_scatter)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*broadcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
  ncclResult_t (*get_version)(int*) = nullptr;
  std::string origin;
};

static Api& api() {
  static Api a;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so", RTLD_NOW | RTLD_NOLOAD);  // torch's, when it is loaded
    a.origin = "process";
    if (!h) { h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD); }
    if (!h) { h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL); a.origin = "/opt/rocm/lib"; }
    if (!h) { a.origin = ""; return; }
#define DBX_SYM(field, name) a.field = reinterpret_cast<decltype(a.field)>(dlsym(h, name))
    DBX_SYM(get_unique_id, "ncclGetUniqueId");
    DBX_SYM(comm_init_rank, "ncclCommInitRank");
    DBX_SYM(comm_init_rank_config, "ncclCommInitRankConfig");
    DBX_SYM(comm_destroy, "ncclCommDestroy");
    DBX_SYM(comm_abort, "ncclCommAbort");
    DBX_SYM(comm_count, "ncclCommCount");
    DBX_SYM(comm_get_async_error, "ncclCommGetAsyncError");
    DBX_SYM(all_reduce, "ncclAllReduce");
    DBX_SYM(reduce_scatter, "ncclReduceScatter");
    DBX_SYM(all_gather, "ncclAllGather");
    DBX_SYM(broadcast, "ncclBroadcast");
    DBX_SYM(group_start, "ncclGroupStart");
    DBX_SYM(group_end, "ncclGroupEnd");
    DBX_SYM(error_string, "ncclGetErrorString");
    DBX_SYM(get_version, "ncclGetVersion");
#undef DBX_SYM
    if (!a.get_unique_id || !a.comm_init_rank || !a.all_reduce || !a.reduce_scatter || !a.all_gather ||
        !a.broadcast || !a.group_start || !a.group_end || !a.comm_destroy)
      a.origin = "";
  });
  return a;
}

static Api& need() {
  Api& a = api();
  if (a.origin.empty()) throw std::runtime_error("native comm: librccl could not be loaded");
  return a;
}

static void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("native comm: ") + what + ": " + hipGetErrorString(e));
}

static void check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) {
    Api& a = api();
    throw std::runtime_error(std::string("native comm: ") + what + " failed: " +
                             (a.error_string ? a.error_string(r) : std::to_string((int)r)));
  }
}

// torch scalar-type codes used by the Python side (ops/_ext-independent small enum)
static ncclDataType_t dtype_of(int code) {
  switch (code) {
    case 0: return ncclFloat32;
    case 1: return ncclBfloat16;
    case 2: return ncclFloat16;
    case 3: return ncclFloat64;
    case 4: return ncclInt32;
    case 5: return ncclInt64;
    case 6: return ncclUint8;
  }
  throw std::invalid_argument("native comm: unsupported dtype code");
}
static ncclRedOp_t op_of(int code) {
  switch (code) {
    case 0: return ncclSum;
    case 1: return ncclAvg;
    case 2: return ncclMax;
    case 3: return ncclMin;
    case 4: return ncclProd;
  }
  throw std::invalid_argument("native comm: unsupported reduction op");
}

struct Communicator {
  ncclComm_t comm = nullptr;  // read / cleared with __atomic builtins where the watchdog thread may abort
  int rank = 0, size = 1, device = 0;
  bool nonblocking = false;
  double timeout_s = 1800.0;  // bound of settle(): the process's collective timeout (comm_set_timeout)
};

static ncclComm_t live(Communicator* c) { return __atomic_load_n(&c->comm, __ATOMIC_ACQUIRE); }

// A non-blocking communicator may answer any call with ncclInProgress (the operation is accepted
// and completes asynchronously): wait for its state to settle, bounded by the communicator's timeout,
// then report it. The wait releases the GIL so the comm watchdog (a Python thread,
// parallel/comm_guard.py) keeps polling and can abort the communicator; an abort ends the wait.
static ncclResult_t settle(Communicator* c, ncclResult_t r) {
  if (r != ncclInProgress || !c || !live(c)) return r;
  Api& a = api();
  if (!a.comm_get_async_error) return ncclSuccess;
  py::gil_scoped_release nogil;
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    ncclComm_t comm = live(c);
    if (!comm) return ncclInvalidUsage;  // aborted meanwhile
    ncclResult_t st = ncclSuccess;
    const ncclResult_t q = a.comm_get_async_error(comm, &st);
    if (q != ncclSuccess) return q;
    if (st != ncclInProgress) return st;
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > c->timeout_s)
      return ncclInProgress;
    usleep(100);
  }
}

}  // namespace comm
}  // namespace dbx

using dbx::comm::Communicator;

void register_comm(py::module& m) {
  using namespace dbx::comm;
  m.def("comm_available", []() { return !api().origin.empty(); });
  m.def("comm_origin", []() { return api().origin; });
  m.def("comm_version", []() {
    Api& a = need();
    int v = 0;
    if (a.get_version) check(a.get_version(&v), "ncclGetVersion");
    return v;
  });
  m.def("comm_unique_id", []() {
    ncclUniqueId id;
    check(need().get_unique_id(&id), "ncclGetUniqueId");
    return py::bytes(id.internal, NCCL_UNIQUE_ID_BYTES);
  });
  // returns an opaque handle (pointer as int); the calling thread's current HIP device is the
  // communicator's device. blocking = 0: ncclCommInitRankConfig returns at once and the caller polls
  // comm_async_error until it leaves ncclInProgress (7) -- so a rank whose peer failed before the
  // rendezvous can abort instead of hanging inside the init (parallel/comm.py). min_ctas / max_ctas
  // (> 0): RCCL's channel (CTA) bounds for this communicator (collective_plan.py).
  m.def("comm_init", [](py::bytes uid, int nranks, int rank, int blocking, int min_ctas, int max_ctas) {
    std::string s = uid;
    if (s.size() != NCCL_UNIQUE_ID_BYTES) throw std::invalid_argument("native comm: bad unique id");
    if (nranks < 1 || rank < 0 || rank >= nranks) throw std::invalid_argument("native comm: bad rank / size");
    ncclUniqueId id;
    std::memcpy(id.internal, s.data(), NCCL_UNIQUE_ID_BYTES);
    auto* c = new Communicator();
    c->rank = rank;
    c->size = nranks;
    c->nonblocking = !blocking;
    if (hipGetDevice(&c->device) != hipSuccess) c->device = 0;
    Api& a = need();
    ncclResult_t r;
    {
      py::gil_scoped_release nogil;  // a blocking init rendezvouses with the other ranks
      if (a.comm_init_rank_config && (!blocking || min_ctas > 0 || max_ctas > 0)) {
        ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
        cfg.blocking = blocking ? 1 : 0;
        if (min_ctas > 0) cfg.minCTAs = min_ctas;
        if (max_ctas > 0) cfg.maxCTAs = max_ctas;
        r = a.comm_init_rank_config(&c->comm, nranks, id, rank, &cfg);
        if (!blocking && r == ncclInProgress) r = ncclSuccess;  // completion: comm_async_error
      } else {
        r = a.comm_init_rank(&c->comm, nranks, id, rank);
      }
    }
    if (r != ncclSuccess) {
      delete c;
      check(r, "ncclCommInitRank");
    }
    return reinterpret_cast<uintptr_t>(c);
  }, py::arg("uid"), py::arg("nranks"), py::arg("rank"), py::arg("blocking") = 1, py::arg("min_ctas") = 0,
     py::arg("max_ctas") = 0);
  m.def("comm_config_supported", []() { return api().comm_init_rank_config != nullptr; });
  m.def("comm_destroy", [](uintptr_t h, bool abort) {
    auto* c = reinterpret_cast<Communicator*>(h);
    if (!c) return;
    Api& a = need();
    if (c->comm) {
      py::gil_scoped_release nogil;
      if (abort && a.comm_abort) a.comm_abort(c->comm);
      else a.comm_destroy(c->comm);
    }
    delete c;
  });
  // failure handling (parallel/comm_guard.py): the communicator's asynchronous error state -- a peer
  // that died or a network / xGMI failure surfaces here while the kernels are still queued -- and an
  // abort that can be issued from the watchdog thread while the main thread is blocked on the
  // device: ncclCommAbort makes the communicator's queued kernels return, so the stream drains
  // (the handle is then inert; a later comm_destroy only frees it)
  m.def("comm_async_error", [](uintptr_t h) -> py::tuple {
    auto* c = reinterpret_cast<Communicator*>(h);
    Api& a = need();
    if (!c || !c->comm) return py::make_tuple(-1, std::string("communicator aborted"));
    if (!a.comm_get_async_error) return py::make_tuple(0, std::string("ncclCommGetAsyncError unavailable"));
    ncclResult_t st = ncclSuccess;
    ncclResult_t r = a.comm_get_async_error(c->comm, &st);
    if (r != ncclSuccess) st = r;
    return py::make_tuple(static_cast<int>(st), std::string(a.error_string ? a.error_string(st) : ""));
  });
  m.def("comm_abort", [](uintptr_t h) {
    auto* c = reinterpret_cast<Communicator*>(h);
    Api& a = need();
    if (!c || !c->comm || !a.comm_abort) return;
    ncclComm_t comm = __atomic_exchange_n(&c->comm, (ncclComm_t) nullptr, __ATOMIC_ACQ_REL);
    if (!comm) return;
    py::gil_scoped_release nogil;
    a.comm_abort(comm);
  });
  m.def("comm_set_timeout", [](uintptr_t h, double s) {
    auto* c = reinterpret_cast<Communicator*>(h);
    if (c && s > 0) c->timeout_s = s;
  });
  m.def("comm_rank", [](uintptr_t h) { return reinterpret_cast<Communicator*>(h)->rank; });
  m.def("comm_size", [](uintptr_t h) { return reinterpret_cast<Communicator*>(h)->size; });
  m.def("comm_all_reduce", [](uintptr_t h, uintptr_t send, uintptr_t recv, size_t count, int dt, int op,
                              uintptr_t stream) {
    auto* c = reinterpret_cast<Communicator*>(h);
    check(settle(c, need().all_reduce(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), count, dtype_of(dt),
                            op_of(op), c->comm, reinterpret_cast<hipStream_t>(stream))),
          "ncclAllReduce");
  });
  // recvcount = elements per rank; send holds size * recvcount
  m.def("comm_reduce_scatter", [](uintptr_t h, uintptr_t send, uintptr_t recv, size_t recvcount, int dt, int op,
                                  uintptr_t stream) {
    auto* c = reinterpret_cast<Communicator*>(h);
    check(settle(c, need().reduce_scatter(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), recvcount,
                                dtype_of(dt), op_of(op), c->comm, reinterpret_cast<hipStream_t>(stream))),
          "ncclReduceScatter");
  });
  m.def("comm_all_gather", [](uintptr_t h, uintptr_t send, uintptr_t recv, size_t sendcount, int dt,
                              uintptr_t stream) {
    auto* c = reinterpret_cast<Communicator*>(h);
    check(settle(c, need().all_gather(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), sendcount,
                            dtype_of(dt), c->comm, reinterpret_cast<hipStream_t>(stream))),
          "ncclAllGather");
  });
  m.def("comm_broadcast", [](uintptr_t h, uintptr_t send, uintptr_t recv, size_t count, int dt, int root,
                             uintptr_t stream) {
    auto* c = reinterpret_cast<Communicator*>(h);
    check(settle(c, need().broadcast(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), count, dtype_of(dt),
                           root, c->comm, reinterpret_cast<hipStream_t>(stream))),
          "ncclBroadcast");
  });
  m.def("comm_group_start", []() { check(need().group_start(), "ncclGroupStart"); });
  m.def("comm_group_end", [](uintptr_t h) {
    check(settle(reinterpret_cast<Communicator*>(h), need().group_end()), "ncclGroupEnd");
  }, py::arg("h") = 0);

  // ---- peer-mapped buffers for the direct xGMI all-reduce (csrc/direct_ar.hip) ----------------
  // handle of the allocation that holds ptr + ptr's offset in it (the caching allocator hands out
  // sub-blocks of larger segments; the peer maps the segment and adds the offset)
  m.def("ipc_handle", [](uintptr_t ptr) -> py::tuple {
    void* base = nullptr;
    size_t size = 0;
    hip_check(hipMemGetAddressRange(&base, &size, reinterpret_cast<void*>(ptr)), "hipMemGetAddressRange");
    hipIpcMemHandle_t h;
    hip_check(hipIpcGetMemHandle(&h, base), "hipIpcGetMemHandle");
    return py::make_tuple(py::bytes(reinterpret_cast<const char*>(&h), sizeof(h)),
                          (long long)(ptr - reinterpret_cast<uintptr_t>(base)));
  });
  m.def("ipc_open", [](py::bytes handle) -> uintptr_t {
    std::string s = handle;
    if (s.size() != sizeof(hipIpcMemHandle_t)) throw std::invalid_argument("ipc_open: bad handle");
    hipIpcMemHandle_t h;
    std::memcpy(&h, s.data(), sizeof(h));
    void* p = nullptr;
    hip_check(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
    return reinterpret_cast<uintptr_t>(p);
  });
  m.def("ipc_close", [](uintptr_t p) { (void)hipIpcCloseMemHandle(reinterpret_cast<void*>(p)); });
  // (flags, gen, err, err_host, err_host_dev): err_host is a pinned host word the kernel mirrors its
  // error bit into, read by dar_host_err without any device sync (the comm watchdog's poll)
  m.def("dar_alloc", [](int grid) -> py::tuple {
    void *f = nullptr, *g = nullptr, *e = nullptr, *eh = nullptr, *ehd = nullptr;
    const int r = dbx_dar_alloc(grid, &f, &g, &e, &eh, &ehd);
    if (r != 0) throw std::runtime_error("dar_alloc failed: hip error " + std::to_string(r));
    return py::make_tuple(reinterpret_cast<uintptr_t>(f), reinterpret_cast<uintptr_t>(g), reinterpret_cast<uintptr_t>(e),
                          reinterpret_cast<uintptr_t>(eh), reinterpret_cast<uintptr_t>(ehd));
  });
  m.def("dar_free", [](uintptr_t f, uintptr_t g, uintptr_t e, uintptr_t eh) {
    dbx_dar_free(reinterpret_cast<void*>(f), reinterpret_cast<void*>(g), reinterpret_cast<void*>(e),
                 reinterpret_cast<void*>(eh));
  }, py::arg("flags"), py::arg("gen"), py::arg("err"), py::arg("err_host") = 0);
  m.def("dar_host_err", [](uintptr_t eh) {
    return eh ? static_cast<int>(*reinterpret_cast<volatile int*>(eh)) : 0;
  });
  m.def("dar_max_ranks", []() { return dbx_dar_max_ranks(); });
  // every rank of one process in one dispatch (tests: co-resident by construction)
  m.def("dar_launch_multi", [](std::vector<uintptr_t> bufs, std::vector<uintptr_t> flags, std::vector<uintptr_t> gens,
                               std::vector<uintptr_t> errs, long long n, int grid, double timeout_s, uintptr_t stream) {
    const int world = (int)bufs.size();
    if ((int)flags.size() != world || (int)gens.size() != world || (int)errs.size() != world)
      throw std::invalid_argument("dar_launch_multi: world");
    std::vector<float*> b(world);
    std::vector<unsigned*> f(world), g(world);
    std::vector<int*> e(world);
    for (int j = 0; j < world; ++j) {
      b[j] = reinterpret_cast<float*>(bufs[j]);
      f[j] = reinterpret_cast<unsigned*>(flags[j]);
      g[j] = reinterpret_cast<unsigned*>(gens[j]);
      e[j] = reinterpret_cast<int*>(errs[j]);
    }
    const int r = dbx_dar_launch_multi(b.data(), f.data(), g.data(), e.data(), n, world, grid, timeout_s,
                                       reinterpret_cast<hipStream_t>(stream));
    if (r != 0) throw std::runtime_error("dar_launch_multi failed: code " + std::to_string(r));
  });
  // the error word (synchronous copy after a device sync by the caller); reset = clear it
  m.def("dar_read_err", [](uintptr_t err, bool reset) {
    int v = 0;
    hip_check(hipMemcpy(&v, reinterpret_cast<void*>(err), sizeof(int), hipMemcpyDeviceToHost), "hipMemcpy");
    if (reset && v) hip_check(hipMemset(reinterpret_cast<void*>(err), 0, sizeof(int)), "hipMemset");
    return v;
  }, py::arg("err"), py::arg("reset") = false);
  m.def("dar_launch", [](std::vector<uintptr_t> bufs, std::vector<uintptr_t> flags, uintptr_t gen, uintptr_t err,
                         long long n, int rank, int world, int grid, double timeout_s, uintptr_t stream,
                         uintptr_t err_host_dev) {
    if ((int)bufs.size() != world || (int)flags.size() != world) throw std::invalid_argument("dar_launch: world");
    std::vector<float*> b(world);
    std::vector<unsigned*> f(world);
    for (int j = 0; j < world; ++j) {
      b[j] = reinterpret_cast<float*>(bufs[j]);
      f[j] = reinterpret_cast<unsigned*>(flags[j]);
    }
    const int r = dbx_dar_launch(b.data(), f.data(), reinterpret_cast<unsigned*>(gen), reinterpret_cast<int*>(err),
                                 reinterpret_cast<int*>(err_host_dev), n, rank, world, grid, timeout_s,
                                 reinterpret_cast<hipStream_t>(stream));
    if (r != 0) throw std::runtime_error("dar_launch failed: code " + std::to_string(r));
  });
}
