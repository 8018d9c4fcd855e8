// RCCL communicator + in-place fp32 all-reduce for the data-parallel gradient sync (aimx.h).
//
// Why not torch.distributed's ProcessGroupNCCL inside the captured train step: its watchdog
// thread polls every collective's end event, and an event recorded during stream capture may not
// be queried (hipErrorCapturedEvent) — the process aborts at random. A communicator of our own,
// driven straight from the step's streams, has no watchdog and captures as plain graph nodes.
//
// RCCL is bound at run time with dlopen/dlsym: the caller passes the path of the RCCL the process
// already has mapped (PyTorch's bundled librccl.so), so the ncclUniqueId exchange, the bootstrap
// and the channels all belong to one RCCL instance.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>

#include "aimx_common.h"

namespace {

struct Rccl {
  void* handle = nullptr;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                             hipStream_t) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*get_version)(int*) = nullptr;
  ncclResult_t (*comm_count)(const ncclComm_t, int*) = nullptr;
};

Rccl g_rccl;
std::mutex g_mu;

template <class F>
bool bind(void* h, const char* name, F& fn) {
  fn = reinterpret_cast<F>(dlsym(h, name));
  return fn != nullptr;
}

// RCCL failures map to a positive code above the hipError_t range the other entry points use
constexpr int kRcclBase = 10000;
inline int rc(ncclResult_t r) { return r == ncclSuccess ? AIMX_OK : kRcclBase + (int)r; }

}  // namespace

extern "C" int aimx_comm_load(const char* rccl_path) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_rccl.handle) return AIMX_OK;
  if (!rccl_path) return AIMX_EARG;
  void* h = dlopen(rccl_path, RTLD_NOW | RTLD_LOCAL);
  if (!h) return AIMX_EARG;
  Rccl r;
  r.handle = h;
  if (!bind(h, "ncclGetUniqueId", r.get_unique_id) || !bind(h, "ncclCommInitRank", r.comm_init_rank) ||
      !bind(h, "ncclAllReduce", r.all_reduce) || !bind(h, "ncclCommDestroy", r.comm_destroy) ||
      !bind(h, "ncclGetVersion", r.get_version) || !bind(h, "ncclCommCount", r.comm_count)) {
    dlclose(h);
    return AIMX_EARG;
  }
  g_rccl = r;
  return AIMX_OK;
}

extern "C" int aimx_comm_unique_id(void* id_out, size_t bytes) {
  if (!g_rccl.handle || !id_out || bytes < sizeof(ncclUniqueId)) return AIMX_EARG;
  ncclUniqueId id;
  const int r = rc(g_rccl.get_unique_id(&id));
  if (r == AIMX_OK) std::memcpy(id_out, &id, sizeof(id));
  return r;
}

extern "C" int aimx_comm_init(void** comm_out, const void* id, size_t bytes, int32_t nranks, int32_t rank) {
  if (!g_rccl.handle || !comm_out || !id || bytes < sizeof(ncclUniqueId) || nranks < 1 || rank < 0 ||
      rank >= nranks)
    return AIMX_EARG;
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  ncclComm_t c = nullptr;
  const int r = rc(g_rccl.comm_init_rank(&c, nranks, uid, rank));
  *comm_out = r == AIMX_OK ? (void*)c : nullptr;
  return r;
}

extern "C" int aimx_comm_allreduce(void* comm, float* buf, int64_t count, int32_t op, aimx_stream_t stream) {
  if (!g_rccl.handle || !comm || count < 0 || (count > 0 && !buf) || (op != 0 && op != 1)) return AIMX_EARG;
  if (count == 0) return AIMX_OK;
  return rc(g_rccl.all_reduce(buf, buf, (size_t)count, ncclFloat32, op == 1 ? ncclAvg : ncclSum, (ncclComm_t)comm,
                              (hipStream_t)stream));
}

extern "C" int aimx_comm_version(int32_t* version_out) {
  if (!g_rccl.handle || !version_out) return AIMX_EARG;
  int v = 0;
  const int r = rc(g_rccl.get_version(&v));
  *version_out = v;
  return r;
}

extern "C" int aimx_comm_count(void* comm, int32_t* nranks_out) {
  if (!g_rccl.handle || !comm || !nranks_out) return AIMX_EARG;
  int n = 0;
  const int r = rc(g_rccl.comm_count((ncclComm_t)comm, &n));
  *nranks_out = n;
  return r;
}

extern "C" int aimx_comm_destroy(void* comm) {
  if (!g_rccl.handle || !comm) return AIMX_EARG;
  return rc(g_rccl.comm_destroy((ncclComm_t)comm));
}
