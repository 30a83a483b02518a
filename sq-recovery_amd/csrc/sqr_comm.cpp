// Data-parallel gradient exchange owned by libsqr: an RCCL communicator created
// and driven here, outside torch's ProcessGroupNCCL.
//
// Why not ProcessGroupNCCL: every collective issued through it becomes a WorkNCCL whose end event
// the PG's watchdog thread polls (hipEventQuery).  When such an event was last recorded inside a
// stream capture (the captured step graph) the poll fails with hipErrorCapturedEvent and the
// watchdog aborts the process — in any capture mode (round-3 GPUTEST: test_dp_graph_gpu).  Here the
// captured graph holds plain RCCL kernels: no Work objects, no event cache, no watchdog.
//
// RCCL is bound at run time (dlopen + dlsym) to the SAME librccl the process already maps (torch's
// bundled copy, soname librccl.so.1): one RCCL runtime per process, no link-time dependency, and
// libsqr still loads on hosts without RCCL (the comm calls then fail with a message).
#include <dlfcn.h>
#include <string.h>

#include <mutex>

#include <rccl/rccl.h>

#include "sqr_common.h"

namespace {

struct Rccl {
  void* handle = nullptr;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                             hipStream_t) = nullptr;
  ncclResult_t (*broadcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*comm_finalize)(ncclComm_t) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*comm_abort)(ncclComm_t) = nullptr;
  ncclResult_t (*comm_async_error)(ncclComm_t, ncclResult_t*) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
  ncclResult_t (*get_version)(int*) = nullptr;
};

Rccl g_rccl;
std::mutex g_rccl_mu;

template <class F>
bool bind(void* h, const char* name, F* out) {
  *out = reinterpret_cast<F>(dlsym(h, name));
  return *out != nullptr;
}

// loaded once per process; later calls with another path keep the first binding
int load_rccl(const char* path) {
  std::lock_guard<std::mutex> lk(g_rccl_mu);
  if (g_rccl.handle) return 0;
  const char* p = (path && path[0]) ? path : "librccl.so.1";
  void* h = dlopen(p, RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    sqr::set_error("comm: dlopen(%s) failed: %s", p, dlerror());
    return SQR_E_UNSUPPORTED;
  }
  Rccl r;
  r.handle = h;
  bool ok = bind(h, "ncclGetUniqueId", &r.get_unique_id) && bind(h, "ncclCommInitRank", &r.comm_init_rank) &&
            bind(h, "ncclAllReduce", &r.all_reduce) && bind(h, "ncclBroadcast", &r.broadcast) &&
            bind(h, "ncclCommDestroy", &r.comm_destroy) &&
            bind(h, "ncclCommAbort", &r.comm_abort) && bind(h, "ncclGetErrorString", &r.error_string) &&
            bind(h, "ncclCommGetAsyncError", &r.comm_async_error) && bind(h, "ncclGetVersion", &r.get_version);
  if (!ok) {
    sqr::set_error("comm: %s lacks an RCCL entry point", p);
    dlclose(h);
    return SQR_E_UNSUPPORTED;
  }
  bind(h, "ncclCommFinalize", &r.comm_finalize);  // optional (RCCL >= 2.14)
  g_rccl = r;
  return 0;
}

int rccl_fail(const char* what, ncclResult_t r) {
  sqr::set_error("comm: %s: %s (ncclResult %d)", what, g_rccl.error_string ? g_rccl.error_string(r) : "?", (int)r);
  return r > 0 ? 1000 + (int)r : SQR_E_UNSUPPORTED;
}

#define SQR_RCCL_LOADED()                                                            \
  do {                                                                               \
    if (!g_rccl.handle) {                                                            \
      ::sqr::set_error("comm: RCCL not loaded (call sqr_comm_load first)");          \
      return SQR_E_UNSUPPORTED;                                                      \
    }                                                                                \
  } while (0)

}  // namespace

struct sqr_comm {
  ncclComm_t nc;
  int nranks, rank;
};

extern "C" int sqr_comm_load(const char* rccl_path, int* version) {
  int rc = load_rccl(rccl_path);
  if (rc) return rc;
  if (version) {
    ncclResult_t r = g_rccl.get_version(version);
    if (r != ncclSuccess) return rccl_fail("ncclGetVersion", r);
  }
  return 0;
}

extern "C" int sqr_comm_unique_id(unsigned char* id_out) {
  SQR_CHECK_ARG(id_out, "comm_unique_id: null output");
  SQR_RCCL_LOADED();
  ncclUniqueId id;
  ncclResult_t r = g_rccl.get_unique_id(&id);
  if (r != ncclSuccess) return rccl_fail("ncclGetUniqueId", r);
  memcpy(id_out, id.internal, SQR_COMM_ID_BYTES);
  return 0;
}

extern "C" int sqr_comm_init_rank(sqr_comm_t* comm, const unsigned char* id, int nranks, int rank) {
  SQR_CHECK_ARG(comm && id, "comm_init_rank: null argument");
  SQR_CHECK_ARG(nranks >= 1 && rank >= 0 && rank < nranks, "comm_init_rank: rank %d of %d", rank, nranks);
  SQR_RCCL_LOADED();
  *comm = nullptr;
  ncclUniqueId uid;
  memcpy(uid.internal, id, SQR_COMM_ID_BYTES);
  ncclComm_t nc = nullptr;
  ncclResult_t r = g_rccl.comm_init_rank(&nc, nranks, uid, rank);
  if (r != ncclSuccess) return rccl_fail("ncclCommInitRank", r);
  *comm = new sqr_comm{nc, nranks, rank};
  return 0;
}

extern "C" int sqr_comm_allreduce_sum_f32(sqr_comm_t comm, float* buf, size_t count, void* stream) {
  SQR_CHECK_ARG(comm, "comm_allreduce: null communicator");
  SQR_CHECK_ARG(buf || count == 0, "comm_allreduce: null buffer");
  if (count == 0) return 0;
  ncclResult_t r = g_rccl.all_reduce(buf, buf, count, ncclFloat32, ncclSum, comm->nc, sqr::as_stream(stream));
  if (r != ncclSuccess) return rccl_fail("ncclAllReduce", r);
  return 0;
}

extern "C" int sqr_comm_broadcast(sqr_comm_t comm, void* buf, size_t bytes, int root, void* stream) {
  SQR_CHECK_ARG(comm, "comm_broadcast: null communicator");
  SQR_CHECK_ARG(buf || bytes == 0, "comm_broadcast: null buffer");
  SQR_CHECK_ARG(root >= 0 && root < comm->nranks, "comm_broadcast: root %d of %d", root, comm->nranks);
  if (bytes == 0) return 0;
  ncclResult_t r = g_rccl.broadcast(buf, buf, bytes, ncclUint8, root, comm->nc, sqr::as_stream(stream));
  if (r != ncclSuccess) return rccl_fail("ncclBroadcast", r);
  return 0;
}

extern "C" int sqr_comm_async_error(sqr_comm_t comm) {
  SQR_CHECK_ARG(comm, "comm_async_error: null communicator");
  ncclResult_t a = ncclSuccess;
  ncclResult_t r = g_rccl.comm_async_error(comm->nc, &a);
  if (r != ncclSuccess) return rccl_fail("ncclCommGetAsyncError", r);
  if (a != ncclSuccess && a != ncclInProgress) return rccl_fail("asynchronous communicator error", a);
  return 0;
}

extern "C" int sqr_comm_destroy(sqr_comm_t comm) {
  if (!comm) return 0;
  int rc = 0;
  if (g_rccl.comm_finalize) {
    ncclResult_t r = g_rccl.comm_finalize(comm->nc);
    if (r != ncclSuccess && r != ncclInProgress) rc = rccl_fail("ncclCommFinalize", r);
  }
  ncclResult_t r = g_rccl.comm_destroy(comm->nc);
  if (r != ncclSuccess && rc == 0) rc = rccl_fail("ncclCommDestroy", r);
  delete comm;
  return rc;
}

// A rank that gives up (host deadline expired, a peer reported an error): ncclCommAbort stops the
// communicator's in-flight kernels and proxy thread instead of waiting for peers that may be gone.
extern "C" int sqr_comm_abort(sqr_comm_t comm) {
  if (!comm) return 0;
  SQR_RCCL_LOADED();
  ncclResult_t r = g_rccl.comm_abort(comm->nc);
  delete comm;
  if (r != ncclSuccess) return rccl_fail("ncclCommAbort", r);
  return 0;
}
