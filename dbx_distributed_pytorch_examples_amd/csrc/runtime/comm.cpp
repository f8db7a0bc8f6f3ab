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
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>

namespace py = pybind11;

namespace dbx {
namespace comm {

struct Api {
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
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
  ncclComm_t comm = nullptr;
  int rank = 0, size = 1, device = 0;
};

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
  // communicator's device
  m.def("comm_init", [](py::bytes uid, int nranks, int rank) {
    std::string s = uid;
    if (s.size() != NCCL_UNIQUE_ID_BYTES) throw std::invalid_argument("native comm: bad unique id");
    if (nranks < 1 || rank < 0 || rank >= nranks) throw std::invalid_argument("native comm: bad rank / size");
    ncclUniqueId id;
    std::memcpy(id.internal, s.data(), NCCL_UNIQUE_ID_BYTES);
    auto* c = new Communicator();
    c->rank = rank;
    c->size = nranks;
    if (hipGetDevice(&c->device) != hipSuccess) c->device = 0;
    ncclResult_t r;
    {
      py::gil_scoped_release nogil;  // init rendezvouses with the other ranks
      r = need().comm_init_rank(&c->comm, nranks, id, rank);
    }
    if (r != ncclSuccess) {
      delete c;
      check(r, "ncclCommInitRank");
    }
    return reinterpret_cast<uintptr_t>(c);
  });
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
    ncclComm_t comm = c->comm;
    c->comm = nullptr;
    py::gil_scoped_release nogil;
    a.comm_abort(comm);
  });
  m.def("comm_rank", [](uintptr_t h) { return reinterpret_cast<Communicator*>(h)->rank; });
  m.def("comm_size", [](uintptr_t h) { return reinterpret_cast<Communicator*>(h)->size; });
  m.def("comm_all_reduce", [](uintptr_t h, uintptr_t send, uintptr_t recv, size_t count, int dt, int op,
                              uintptr_t stream) {
    auto* c = reinterpret_cast<Communicator*>(h);
    check(need().all_reduce(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), count, dtype_of(dt),
                            op_of(op), c->comm, reinterpret_cast<hipStream_t>(stream)),
          "ncclAllReduce");
  });
  // recvcount = elements per rank; send holds size * recvcount
  m.def("comm_reduce_scatter", [](uintptr_t h, uintptr_t send, uintptr_t recv, size_t recvcount, int dt, int op,
                                  uintptr_t stream) {
    auto* c = reinterpret_cast<Communicator*>(h);
    check(need().reduce_scatter(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), recvcount,
                                dtype_of(dt), op_of(op), c->comm, reinterpret_cast<hipStream_t>(stream)),
          "ncclReduceScatter");
  });
  m.def("comm_all_gather", [](uintptr_t h, uintptr_t send, uintptr_t recv, size_t sendcount, int dt,
                              uintptr_t stream) {
    auto* c = reinterpret_cast<Communicator*>(h);
    check(need().all_gather(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), sendcount,
                            dtype_of(dt), c->comm, reinterpret_cast<hipStream_t>(stream)),
          "ncclAllGather");
  });
  m.def("comm_broadcast", [](uintptr_t h, uintptr_t send, uintptr_t recv, size_t count, int dt, int root,
                             uintptr_t stream) {
    auto* c = reinterpret_cast<Communicator*>(h);
    check(need().broadcast(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), count, dtype_of(dt),
                           root, c->comm, reinterpret_cast<hipStream_t>(stream)),
          "ncclBroadcast");
  });
  m.def("comm_group_start", []() { check(need().group_start(), "ncclGroupStart"); });
  m.def("comm_group_end", []() { check(need().group_end(), "ncclGroupEnd"); });
}
