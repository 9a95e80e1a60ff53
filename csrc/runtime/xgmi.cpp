// Host side of the xGMI all-reduce (csrc/kernels/xgmi.hip): the IPC workspace.
//
// Each rank allocates one data allocation (two buffers, by round parity) and
// one flag array in UNCACHED device memory (hipDeviceMallocUncached: peers
// poll it across xGMI, so it must never sit stale in an L2), exports both
// with hipIpcGetMemHandle, and maps every peer's pair with
// hipIpcOpenMemHandle.  An abort word lives in mapped pinned host memory: the
// elastic watchdog sets it from the CPU and every spinning workgroup sees it.
#include <hip/hip_runtime.h>

#include <cstring>
#include <vector>

#include "../include/xgmi_layout.h"

using edl_xgmi::kFlagBytes;
using edl_xgmi::kMaxRanks;
using edl_xgmi::kStatusWords;

namespace {

struct Workspace {
  int device = 0;
  size_t data_bytes = 0;  // per parity buffer
  char* data = nullptr;   // 2 * data_bytes
  void* flags = nullptr;
  int* abort_host = nullptr;
  int* abort_dev = nullptr;
  int* status = nullptr;       // device view of status_host (kStatusWords ints)
  int* status_host = nullptr;
  int nranks = 1, rank = 0;
  std::vector<char*> peer_data;    // nranks (own included)
  std::vector<void*> peer_flags;   // nranks
};

}  // namespace

extern "C" {

int edl_xgmi_ws_create(int device, uint64_t data_bytes, void** out) {
  if (hipSetDevice(device) != hipSuccess) return -1;
  auto* w = new Workspace();
  w->device = device;
  w->data_bytes = (data_bytes + 255) & ~uint64_t(255);
  hipError_t e = hipMalloc((void**)&w->data, 2 * w->data_bytes);
  if (e == hipSuccess) e = hipExtMallocWithFlags(&w->flags, kFlagBytes, hipDeviceMallocUncached);
  if (e == hipSuccess) e = hipMemset(w->flags, 0, kFlagBytes);
  if (e == hipSuccess) e = hipHostMalloc((void**)&w->abort_host, sizeof(int), hipHostMallocMapped);
  if (e == hipSuccess) {
    *w->abort_host = 0;
    e = hipHostGetDevicePointer((void**)&w->abort_dev, w->abort_host, 0);
  }
  // status word in mapped pinned host memory: readable without a hipMemcpy, which
  // would go through the legacy NULL stream and wait for every blocking stream
  // (e.g. a CU-masked snapshot copy in flight)
  if (e == hipSuccess) e = hipHostMalloc((void**)&w->status_host, kStatusWords * sizeof(int), hipHostMallocMapped);
  if (e == hipSuccess) {
    memset(w->status_host, 0, kStatusWords * sizeof(int));
    e = hipHostGetDevicePointer((void**)&w->status, w->status_host, 0);
  }
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    delete w;
    return (int)e;
  }
  *out = w;
  return 0;
}

// out: 2 * 64 bytes (data handle, flag handle)
int edl_xgmi_ws_handles(void* ws, char* out) {
  auto* w = (Workspace*)ws;
  hipIpcMemHandle_t hd, hf;
  hipError_t e = hipIpcGetMemHandle(&hd, w->data);
  if (e == hipSuccess) e = hipIpcGetMemHandle(&hf, w->flags);
  if (e != hipSuccess) return (int)e;
  static_assert(sizeof(hipIpcMemHandle_t) == 64, "IPC handle size");
  memcpy(out, &hd, 64);
  memcpy(out + 64, &hf, 64);
  return 0;
}

// handles: nranks * 128 bytes in rank order (this rank's entry is ignored)
int edl_xgmi_ws_open(void* ws, int nranks, int rank, const char* handles) {
  auto* w = (Workspace*)ws;
  if (nranks < 1 || nranks > kMaxRanks) return (int)hipErrorInvalidValue;
  hipSetDevice(w->device);
  w->nranks = nranks;
  w->rank = rank;
  w->peer_data.assign(nranks, nullptr);
  w->peer_flags.assign(nranks, nullptr);
  for (int p = 0; p < nranks; ++p) {
    if (p == rank) {
      w->peer_data[p] = w->data;
      w->peer_flags[p] = w->flags;
      continue;
    }
    hipIpcMemHandle_t hd, hf;
    memcpy(&hd, handles + 128 * p, 64);
    memcpy(&hf, handles + 128 * p + 64, 64);
    void* d = nullptr;
    void* f = nullptr;
    hipError_t e = hipIpcOpenMemHandle(&d, hd, hipIpcMemLazyEnablePeerAccess);
    if (e == hipSuccess) e = hipIpcOpenMemHandle(&f, hf, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) return (int)e;
    w->peer_data[p] = (char*)d;
    w->peer_flags[p] = f;
  }
  return 0;
}

// data: 2*nranks pointers (rank-major, parity minor); flags: nranks pointers
int edl_xgmi_ws_ptrs(void* ws, void** data, void** flags) {
  auto* w = (Workspace*)ws;
  for (int p = 0; p < w->nranks; ++p) {
    data[2 * p] = w->peer_data[p];
    data[2 * p + 1] = w->peer_data[p] + w->data_bytes;
    flags[p] = w->peer_flags[p];
  }
  return 0;
}

uint64_t edl_xgmi_ws_bytes(void* ws) { return ((Workspace*)ws)->data_bytes; }
int* edl_xgmi_ws_abort_dev(void* ws) { return ((Workspace*)ws)->abort_dev; }
int* edl_xgmi_ws_status_dev(void* ws) { return ((Workspace*)ws)->status; }

void edl_xgmi_ws_set_abort(void* ws, int v) {
  __atomic_store_n(((Workspace*)ws)->abort_host, v, __ATOMIC_SEQ_CST);
}

// status word (0 = ok, 1 = a barrier gave up); valid once the caller has
// synchronised with the collectives it asks about
int edl_xgmi_ws_status(void* ws) {
  auto* w = (Workspace*)ws;
  return __atomic_load_n(w->status_host, __ATOMIC_ACQUIRE);
}

// the whole status record (kStatusWords ints, layout in xgmi_layout.h)
int edl_xgmi_ws_status_detail(void* ws, int* out) {
  auto* w = (Workspace*)ws;
  if (__atomic_load_n(w->status_host, __ATOMIC_ACQUIRE) == 0) {
    memset(out, 0, kStatusWords * sizeof(int));
    return 0;
  }
  for (int i = 0; i < kStatusWords; ++i) out[i] = __atomic_load_n(w->status_host + i, __ATOMIC_RELAXED);
  return out[0];
}

int edl_xgmi_ws_destroy(void* ws) {
  auto* w = (Workspace*)ws;
  if (!w) return 0;
  hipSetDevice(w->device);
  for (int p = 0; p < (int)w->peer_data.size(); ++p) {
    if (p == w->rank) continue;
    if (w->peer_data[p]) hipIpcCloseMemHandle(w->peer_data[p]);
    if (w->peer_flags[p]) hipIpcCloseMemHandle(w->peer_flags[p]);
  }
  if (w->data) hipFree(w->data);
  if (w->flags) hipFree(w->flags);
  if (w->status_host) hipHostFree(w->status_host);
  if (w->abort_host) hipHostFree(w->abort_host);
  delete w;
  return 0;
}

// ---- registered buffers (e.g. the flat gradient buffer, mapped by every peer) ----
// IPC handles name whole allocations, so a tensor inside a caching-allocator
// segment is exported as (handle of its segment, byte offset).
int edl_xgmi_buf_handle(void* ptr, char* out_handle, uint64_t* out_offset, uint64_t* out_segment_bytes) {
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  hipError_t e = hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)ptr);
  if (e != hipSuccess) return (int)e;
  hipIpcMemHandle_t h;
  e = hipIpcGetMemHandle(&h, (void*)base);
  if (e != hipSuccess) return (int)e;
  memcpy(out_handle, &h, sizeof(h));
  *out_offset = (uint64_t)((char*)ptr - (char*)base);
  *out_segment_bytes = (uint64_t)size;
  return 0;
}

int edl_xgmi_buf_open(int device, const char* handle, void** out) {
  hipSetDevice(device);
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  return (int)hipIpcOpenMemHandle(out, h, hipIpcMemLazyEnablePeerAccess);
}

int edl_xgmi_buf_close(int device, void* p) {
  hipSetDevice(device);
  return (int)hipIpcCloseMemHandle(p);
}

}  // extern "C"
