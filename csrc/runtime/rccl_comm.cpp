// Native RCCL communicator manager.
//
// Why not only ProcessGroupNCCL: an elastic job must be able to give up on a
// communicator at ANY point — while it is being created (a peer died during
// the epoch's bootstrap) as well as inside a collective.  This manager
//   * creates communicators NON-BLOCKING (ncclConfig_t.blocking = 0) and polls
//     ncclCommGetAsyncError, so creation can be abandoned by an abort flag or a
//     deadline instead of blocking inside C++ (with the Python GIL held);
//   * exposes ncclCommAbort for the watchdog (kernels stuck on a dead peer exit);
//   * shrinks a communicator to the surviving ranks with ncclCommShrink when
//     the loaded RCCL has it (resolved at run time), avoiding a full re-init;
//   * launches collectives on the caller's HIP stream (no extra copies).
//
// RCCL is not linked at build time: the process already holds torch's
// librccl.so.1 (same SONAME as /opt/rocm's), so the symbols are taken from the
// loaded copy with dlopen(RTLD_NOLOAD) — one RCCL per process, and optional
// entry points (ncclCommShrink) can be probed instead of failing at load.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <cstring>
#include <thread>

namespace {

struct Api {
  bool ok = false;
  decltype(&ncclGetUniqueId) getUniqueId = nullptr;
  decltype(&ncclCommInitRankConfig) initRankConfig = nullptr;
  decltype(&ncclCommGetAsyncError) getAsyncError = nullptr;
  decltype(&ncclCommAbort) abort = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclCommFinalize) finalize = nullptr;
  decltype(&ncclCommSplit) split = nullptr;
  decltype(&ncclAllReduce) allReduce = nullptr;
  decltype(&ncclBroadcast) broadcast = nullptr;
  decltype(&ncclReduceScatter) reduceScatter = nullptr;
  decltype(&ncclAllGather) allGather = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclGroupStart) groupStart = nullptr;
  decltype(&ncclGroupEnd) groupEnd = nullptr;
  decltype(&ncclGetErrorString) errorString = nullptr;
  decltype(&ncclGetVersion) getVersion = nullptr;
  // optional (newer RCCL only)
  ncclResult_t (*shrink)(ncclComm_t, int*, int, ncclComm_t*, ncclConfig_t*, int) = nullptr;
};

Api g_api;
std::atomic<int> g_loaded{0};

template <typename T>
void sym(void* h, const char* name, T& fn) {
  fn = reinterpret_cast<T>(dlsym(h, name));
}

const Api& api() {
  if (g_loaded.load(std::memory_order_acquire)) return g_api;
  void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);  // torch's copy, if loaded
  if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
  if (h) {
    sym(h, "ncclGetUniqueId", g_api.getUniqueId);
    sym(h, "ncclCommInitRankConfig", g_api.initRankConfig);
    sym(h, "ncclCommGetAsyncError", g_api.getAsyncError);
    sym(h, "ncclCommAbort", g_api.abort);
    sym(h, "ncclCommDestroy", g_api.destroy);
    sym(h, "ncclCommFinalize", g_api.finalize);
    sym(h, "ncclCommSplit", g_api.split);
    sym(h, "ncclAllReduce", g_api.allReduce);
    sym(h, "ncclBroadcast", g_api.broadcast);
    sym(h, "ncclReduceScatter", g_api.reduceScatter);
    sym(h, "ncclAllGather", g_api.allGather);
    sym(h, "ncclSend", g_api.send);
    sym(h, "ncclRecv", g_api.recv);
    sym(h, "ncclGroupStart", g_api.groupStart);
    sym(h, "ncclGroupEnd", g_api.groupEnd);
    sym(h, "ncclGetErrorString", g_api.errorString);
    sym(h, "ncclGetVersion", g_api.getVersion);
    sym(h, "ncclCommShrink", g_api.shrink);
    g_api.ok = g_api.getUniqueId && g_api.initRankConfig && g_api.getAsyncError && g_api.abort &&
               g_api.destroy && g_api.allReduce && g_api.broadcast && g_api.reduceScatter && g_api.allGather &&
               g_api.send && g_api.recv && g_api.groupStart && g_api.groupEnd;
  }
  g_loaded.store(1, std::memory_order_release);
  return g_api;
}

// Poll a non-blocking communicator until it is ready, failed, aborted or late.
// Returns 0 on success, >0 an ncclResult_t, -1 aborted by flag, -2 timed out.
int wait_ready(ncclComm_t c, const volatile int* abort_flag, double timeout_s) {
  const auto t_end = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
  while (true) {
    ncclResult_t st = ncclSuccess;
    ncclResult_t r = g_api.getAsyncError(c, &st);
    if (r != ncclSuccess) return (int)r;
    if (st == ncclSuccess) return 0;
    if (st != ncclInProgress) return (int)st;
    if (abort_flag && *abort_flag) return -1;
    if (std::chrono::steady_clock::now() > t_end) return -2;
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
}

ncclConfig_t nonblocking_config() {
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;
  return cfg;
}

}  // namespace

extern "C" {

// 1 if RCCL could be resolved; version in *version (e.g. 22606), shrink support in *has_shrink.
int edl_rccl_available(int* version, int* has_shrink) {
  const Api& a = api();
  if (version) {
    *version = 0;
    if (a.getVersion) a.getVersion(version);
  }
  if (has_shrink) *has_shrink = a.shrink != nullptr;
  return a.ok ? 1 : 0;
}

const char* edl_rccl_error_string(int code) {
  const Api& a = api();
  if (code == -1) return "aborted";
  if (code == -2) return "timed out";
  return a.errorString ? a.errorString((ncclResult_t)code) : "unknown";
}

// out: NCCL_UNIQUE_ID_BYTES (128) bytes
int edl_rccl_unique_id(char* out) {
  const Api& a = api();
  if (!a.ok) return -3;
  ncclUniqueId id;
  ncclResult_t r = a.getUniqueId(&id);
  if (r != ncclSuccess) return (int)r;
  memcpy(out, id.internal, NCCL_UNIQUE_ID_BYTES);
  return 0;
}

// Non-blocking communicator creation, abandoned when *abort_flag becomes
// non-zero or after timeout_s (the half-built communicator is then aborted).
int edl_rccl_init(const char* id_bytes, int nranks, int rank, int device, const int* abort_flag, double timeout_s,
                  void** out) {
  const Api& a = api();
  if (!a.ok) return -3;
  if (hipSetDevice(device) != hipSuccess) return -4;
  ncclUniqueId id;
  memcpy(id.internal, id_bytes, NCCL_UNIQUE_ID_BYTES);
  ncclConfig_t cfg = nonblocking_config();
  ncclComm_t c = nullptr;
  ncclResult_t r = a.initRankConfig(&c, nranks, id, rank, &cfg);
  if (r != ncclSuccess && r != ncclInProgress) return (int)r;
  int st = wait_ready(c, (const volatile int*)abort_flag, timeout_s);
  if (st != 0) {
    a.abort(c);
    return st;
  }
  *out = c;
  return 0;
}

// Drop `nexclude` ranks (dead peers) without a full re-init (RCCL >= 2.27).
// Returns -5 when the loaded RCCL has no ncclCommShrink.
int edl_rccl_shrink(void* comm, const int* exclude, int nexclude, int abort_mode, const int* abort_flag,
                    double timeout_s, void** out) {
  const Api& a = api();
  if (!a.shrink) return -5;
  ncclConfig_t cfg = nonblocking_config();
  ncclComm_t nc = nullptr;
  // flag 0x01 = NCCL_SHRINK_ABORT: the parent may have collectives stuck on a dead rank
  ncclResult_t r = a.shrink((ncclComm_t)comm, const_cast<int*>(exclude), nexclude, &nc, &cfg,
                            abort_mode ? 0x01 : 0x00);
  if (r != ncclSuccess && r != ncclInProgress) return (int)r;
  int st = wait_ready(nc, (const volatile int*)abort_flag, timeout_s);
  if (st != 0) {
    a.abort(nc);
    return st;
  }
  *out = nc;
  return 0;
}

// ncclCommAbort: safe from any thread; kernels blocked on a dead peer return.
int edl_rccl_abort(void* comm) {
  const Api& a = api();
  return comm && a.abort ? (int)a.abort((ncclComm_t)comm) : 0;
}

int edl_rccl_destroy(void* comm) {
  const Api& a = api();
  if (!comm) return 0;
  if (a.finalize) {
    ncclResult_t r = a.finalize((ncclComm_t)comm);
    if (r == ncclSuccess || r == ncclInProgress) wait_ready((ncclComm_t)comm, nullptr, 30.0);
  }
  return (int)a.destroy((ncclComm_t)comm);
}

// ncclSuccess / ncclInProgress / an error raised asynchronously (e.g. a peer vanished)
int edl_rccl_async_error(void* comm) {
  const Api& a = api();
  ncclResult_t st = ncclSuccess;
  ncclResult_t r = a.getAsyncError((ncclComm_t)comm, &st);
  return r != ncclSuccess ? (int)r : (int)st;
}

// Collectives on the caller's stream.  dtype / op use the ncclDataType_t /
// ncclRedOp_t codes (ncclFloat32 = 7, ncclBfloat16 = 9, ncclSum = 0, ...).
// With non-blocking communicators a call may return ncclInProgress while the
// enqueue completes; wait for it here so the caller sees plain success.
static int finish(ncclComm_t c, ncclResult_t r) {
  if (r == ncclInProgress) return wait_ready(c, nullptr, 600.0);
  return (int)r;
}

int edl_rccl_all_reduce(void* comm, const void* send, void* recv, size_t count, int dtype, int op,
                        hipStream_t stream) {
  ncclComm_t c = (ncclComm_t)comm;
  return finish(c, api().allReduce(send, recv, count, (ncclDataType_t)dtype, (ncclRedOp_t)op, c, stream));
}

int edl_rccl_broadcast(void* comm, const void* send, void* recv, size_t count, int dtype, int root,
                       hipStream_t stream) {
  ncclComm_t c = (ncclComm_t)comm;
  return finish(c, api().broadcast(send, recv, count, (ncclDataType_t)dtype, root, c, stream));
}

int edl_rccl_reduce_scatter(void* comm, const void* send, void* recv, size_t recv_count, int dtype, int op,
                            hipStream_t stream) {
  ncclComm_t c = (ncclComm_t)comm;
  return finish(c, api().reduceScatter(send, recv, recv_count, (ncclDataType_t)dtype, (ncclRedOp_t)op, c, stream));
}

int edl_rccl_all_gather(void* comm, const void* send, void* recv, size_t send_count, int dtype,
                        hipStream_t stream) {
  ncclComm_t c = (ncclComm_t)comm;
  return finish(c, api().allGather(send, recv, send_count, (ncclDataType_t)dtype, c, stream));
}

// Point-to-point: a batch of sends/recvs issued as one group (no ordering deadlock).
int edl_rccl_sendrecv(void* comm, int n, const int* is_send, void* const* bufs, const size_t* counts,
                      const int* peers, int dtype, hipStream_t stream) {
  const Api& a = api();
  ncclComm_t c = (ncclComm_t)comm;
  ncclResult_t r = a.groupStart();
  if (r != ncclSuccess) return (int)r;
  for (int i = 0; i < n && r == ncclSuccess; ++i) {
    r = is_send[i] ? a.send(bufs[i], counts[i], (ncclDataType_t)dtype, peers[i], c, stream)
                   : a.recv(bufs[i], counts[i], (ncclDataType_t)dtype, peers[i], c, stream);
  }
  ncclResult_t e = a.groupEnd();
  if (r != ncclSuccess) return (int)r;
  return finish(c, e);
}

}  // extern "C"
