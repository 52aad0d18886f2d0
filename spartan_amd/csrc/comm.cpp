// libspx.so -- cross-GPU collectives behind include/spx.h, on RCCL over xGMI.
//
// The reference moves every partial between workers as pickled ZeroMQ
// point-to-point messages merged at the owner (spartan/array/distarray.py:
// 370-421 update -> blob_ctx.update -> worker.update -> tile.merge,
// spartan/expr/map.py:326-328 for the dot partials); here each of those
// exchange steps is one RCCL collective enqueued on the caller's HIP stream,
// so it is ordered with the kernels around it without host synchronisation.
//
// RCCL is opened at run time (dlopen) by spx_comm_load, so libspx.so loads
// and its compute entry points run in processes that never communicate (and
// in the CPU-only test container).  The Python side passes the path of the
// RCCL that PyTorch-ROCm itself loaded, so one RCCL (and one HIP runtime)
// serves the process.  A communicator is created from a unique id that rank
// 0 makes and the host control plane (torch.distributed gloo store) hands to
// every rank.
#include <dlfcn.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>

#include "../../include/spx.h"

extern "C" int spx_comm_set_error(const char* msg);  // spx.hip: thread-local error text

namespace {

// The slice of rccl.h this file needs (RCCL 2.x ABI, ROCm 7.2:
// /opt/rocm/include/rccl/rccl.h).  Declared here so the library does not
// link against librccl.
typedef struct ncclComm* ncclComm_t;
typedef struct { char internal[128]; } ncclUniqueId;
typedef int ncclResult_t;  // 0 = ncclSuccess
enum { nccl_int8 = 0, nccl_uint8 = 1, nccl_int32 = 2, nccl_int64 = 4, nccl_float32 = 7, nccl_float64 = 8 };
enum { nccl_sum = 0, nccl_prod = 1, nccl_max = 2, nccl_min = 3 };

struct Rccl {
  void* h = nullptr;
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*AllReduce)(const void*, void*, size_t, int, int, ncclComm_t, void*) = nullptr;
  ncclResult_t (*ReduceScatter)(const void*, void*, size_t, int, int, ncclComm_t, void*) = nullptr;
  ncclResult_t (*AllGather)(const void*, void*, size_t, int, ncclComm_t, void*) = nullptr;
  ncclResult_t (*Broadcast)(const void*, void*, size_t, int, int, ncclComm_t, void*) = nullptr;
  ncclResult_t (*Reduce)(const void*, void*, size_t, int, int, int, ncclComm_t, void*) = nullptr;
  ncclResult_t (*Send)(const void*, size_t, int, int, ncclComm_t, void*) = nullptr;
  ncclResult_t (*Recv)(void*, size_t, int, int, ncclComm_t, void*) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
};

Rccl g_rccl;
std::mutex g_mu;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  spx_comm_set_error(buf);
  return code;
}

int rc_check(ncclResult_t r, const char* what) {
  if (r == 0) return SPX_OK;
  const char* msg = g_rccl.GetErrorString ? g_rccl.GetErrorString(r) : "?";
  return fail(SPX_EHIP, "%s failed: rccl error %d (%s)", what, (int)r, msg);
}

bool nccl_dtype(int dt, int* out) {
  switch (dt) {
    case SPX_BOOL: *out = nccl_uint8; return true;
    case SPX_I32: *out = nccl_int32; return true;
    case SPX_I64: *out = nccl_int64; return true;
    case SPX_F32: *out = nccl_float32; return true;
    case SPX_F64: *out = nccl_float64; return true;
    default: return false;
  }
}

bool nccl_op(int op, int* out) {
  switch (op) {
    case SPX_OP_SUM: *out = nccl_sum; return true;
    case SPX_OP_MIN: *out = nccl_min; return true;
    case SPX_OP_MAX: *out = nccl_max; return true;
    default: return false;
  }
}

#define NEED_LOADED()                                                                    \
  do {                                                                                   \
    if (!g_rccl.h) return fail(SPX_EINVAL, "RCCL not loaded: call spx_comm_load first"); \
  } while (0)

#define DT_OP(dt, op)                                                            \
  int ndt_ = 0, nop_ = 0;                                                        \
  if (!nccl_dtype(dt, &ndt_)) return fail(SPX_EINVAL, "bad dtype %d", (int)(dt)); \
  if (!nccl_op(op, &nop_)) return fail(SPX_EINVAL, "bad op %d", (int)(op));

}  // namespace

extern "C" int spx_comm_load(const char* rccl_path) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_rccl.h) return SPX_OK;
  const char* path = (rccl_path && *rccl_path) ? rccl_path : "librccl.so.1";
  void* h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
  if (!h) return fail(SPX_ENOTSUP, "spx_comm_load: dlopen(%s): %s", path, dlerror());
  Rccl r;
  r.h = h;
#define SYM(field, name)                                                               \
  r.field = reinterpret_cast<decltype(r.field)>(dlsym(h, name));                       \
  if (!r.field) {                                                                      \
    dlclose(h);                                                                        \
    return fail(SPX_ENOTSUP, "spx_comm_load: %s has no symbol %s", path, name);        \
  }
  SYM(GetUniqueId, "ncclGetUniqueId")
  SYM(CommInitRank, "ncclCommInitRank")
  SYM(CommDestroy, "ncclCommDestroy")
  SYM(AllReduce, "ncclAllReduce")
  SYM(ReduceScatter, "ncclReduceScatter")
  SYM(AllGather, "ncclAllGather")
  SYM(Broadcast, "ncclBroadcast")
  SYM(Reduce, "ncclReduce")
  SYM(Send, "ncclSend")
  SYM(Recv, "ncclRecv")
  SYM(GroupStart, "ncclGroupStart")
  SYM(GroupEnd, "ncclGroupEnd")
  SYM(GetErrorString, "ncclGetErrorString")
#undef SYM
  g_rccl = r;
  return SPX_OK;
}

extern "C" int spx_comm_unique_id(uint8_t* out, int64_t nbytes) {
  NEED_LOADED();
  if (!out || nbytes < (int64_t)sizeof(ncclUniqueId))
    return fail(SPX_EINVAL, "spx_comm_unique_id: buffer of %lld < %zu bytes", (long long)nbytes, sizeof(ncclUniqueId));
  ncclUniqueId id;
  int rc = rc_check(g_rccl.GetUniqueId(&id), "ncclGetUniqueId");
  if (rc) return rc;
  memcpy(out, id.internal, sizeof(id.internal));
  return SPX_OK;
}

extern "C" int spx_comm_init(const uint8_t* unique_id, int64_t nbytes, int rank, int world, void** comm_out) {
  NEED_LOADED();
  if (!unique_id || nbytes < (int64_t)sizeof(ncclUniqueId) || !comm_out)
    return fail(SPX_EINVAL, "spx_comm_init: bad unique id / output");
  if (world < 1 || rank < 0 || rank >= world) return fail(SPX_EINVAL, "spx_comm_init: rank %d of %d", rank, world);
  ncclUniqueId id;
  memcpy(id.internal, unique_id, sizeof(id.internal));
  ncclComm_t c = nullptr;
  int rc = rc_check(g_rccl.CommInitRank(&c, world, id, rank), "ncclCommInitRank");
  if (rc) return rc;
  *comm_out = c;
  return SPX_OK;
}

extern "C" int spx_comm_destroy(void* comm) {
  NEED_LOADED();
  if (!comm) return SPX_OK;
  return rc_check(g_rccl.CommDestroy((ncclComm_t)comm), "ncclCommDestroy");
}

extern "C" int spx_allreduce(void* comm, const void* send, void* recv, int64_t count, int dtype, int op,
                             void* stream) {
  NEED_LOADED();
  DT_OP(dtype, op);
  if (count < 0 || !comm) return fail(SPX_EINVAL, "spx_allreduce: bad count / comm");
  if (count == 0) return SPX_OK;
  return rc_check(g_rccl.AllReduce(send, recv, (size_t)count, ndt_, nop_, (ncclComm_t)comm, stream), "ncclAllReduce");
}

extern "C" int spx_reduce_scatter(void* comm, const void* send, void* recv, int64_t recvcount, int dtype, int op,
                                  void* stream) {
  NEED_LOADED();
  DT_OP(dtype, op);
  if (recvcount < 0 || !comm) return fail(SPX_EINVAL, "spx_reduce_scatter: bad count / comm");
  if (recvcount == 0) return SPX_OK;
  return rc_check(g_rccl.ReduceScatter(send, recv, (size_t)recvcount, ndt_, nop_, (ncclComm_t)comm, stream),
                  "ncclReduceScatter");
}

extern "C" int spx_allgather(void* comm, const void* send, void* recv, int64_t sendcount, int dtype, void* stream) {
  NEED_LOADED();
  int ndt = 0;
  if (!nccl_dtype(dtype, &ndt)) return fail(SPX_EINVAL, "spx_allgather: bad dtype %d", dtype);
  if (sendcount < 0 || !comm) return fail(SPX_EINVAL, "spx_allgather: bad count / comm");
  if (sendcount == 0) return SPX_OK;
  return rc_check(g_rccl.AllGather(send, recv, (size_t)sendcount, ndt, (ncclComm_t)comm, stream), "ncclAllGather");
}

extern "C" int spx_broadcast(void* comm, const void* send, void* recv, int64_t count, int dtype, int root,
                             void* stream) {
  NEED_LOADED();
  int ndt = 0;
  if (!nccl_dtype(dtype, &ndt)) return fail(SPX_EINVAL, "spx_broadcast: bad dtype %d", dtype);
  if (count < 0 || !comm) return fail(SPX_EINVAL, "spx_broadcast: bad count / comm");
  if (count == 0) return SPX_OK;
  return rc_check(g_rccl.Broadcast(send, recv, (size_t)count, ndt, root, (ncclComm_t)comm, stream), "ncclBroadcast");
}

extern "C" int spx_reduce(void* comm, const void* send, void* recv, int64_t count, int dtype, int op, int root,
                          void* stream) {
  NEED_LOADED();
  DT_OP(dtype, op);
  if (count < 0 || !comm) return fail(SPX_EINVAL, "spx_reduce: bad count / comm");
  if (count == 0) return SPX_OK;
  return rc_check(g_rccl.Reduce(send, recv, (size_t)count, ndt_, nop_, root, (ncclComm_t)comm, stream),
                  "ncclReduce");
}

extern "C" int spx_sendrecv(void* comm, int nsend, const void* const* sbufs, const int64_t* sbytes,
                            const int* speers, int nrecv, void* const* rbufs, const int64_t* rbytes,
                            const int* rpeers, void* stream) {
  NEED_LOADED();
  if (!comm || nsend < 0 || nrecv < 0) return fail(SPX_EINVAL, "spx_sendrecv: bad arguments");
  if (nsend + nrecv == 0) return SPX_OK;
  int rc = rc_check(g_rccl.GroupStart(), "ncclGroupStart");
  if (rc) return rc;
  for (int i = 0; i < nsend && !rc; ++i)
    if (sbytes[i] > 0)
      rc = rc_check(g_rccl.Send(sbufs[i], (size_t)sbytes[i], nccl_uint8, speers[i], (ncclComm_t)comm, stream),
                    "ncclSend");
  for (int i = 0; i < nrecv && !rc; ++i)
    if (rbytes[i] > 0)
      rc = rc_check(g_rccl.Recv(rbufs[i], (size_t)rbytes[i], nccl_uint8, rpeers[i], (ncclComm_t)comm, stream),
                    "ncclRecv");
  int rc2 = rc_check(g_rccl.GroupEnd(), "ncclGroupEnd");
  return rc ? rc : rc2;
}
