// Custom xGMI all-reduce for one MI355X node.
//
// Every rank owns an IPC-exported workspace (two data buffers for round
// parity + a flag array in uncached memory) that all peers map
// (csrc/runtime/xgmi.cpp).  A node's GPUs are fully connected point-to-point
// (7 xGMI links each), so instead of a ring every rank reads every peer
// directly:
//   * one-shot (small messages): each workgroup copies its slice of the input
//     into the rank's own buffer, signals that slice to all peers, waits for
//     the peers' signals and sums the slice from all N buffers (N-1 remote
//     reads in parallel over N-1 links) straight into the output;
//   * two-shot (large messages): reduce-scatter — rank r sums ITS chunk from
//     all peers into its own buffer — then all-gather — every rank copies
//     chunk p from rank p.  Each byte crosses a link twice in total, spread
//     over all 7 links, instead of 2(N-1)/N hops around one ring.
// Synchronisation is per workgroup (workgroup b of every rank handles the
// same slice), with system-scope release/acquire on the flags; the round
// number makes flags monotone, and two data buffers by round parity make a
// buffer safe to overwrite one round later.  Every spin is bounded: it gives
// up when a host-mapped abort word is set (the elastic watchdog) or after a
// deadline, records an error and exits — a dead peer never hangs the GPU.
#include "../include/xgmi_layout.h"
#include "common.h"

using namespace edl;

namespace {

constexpr int XG_MAX_RANKS = edl_xgmi::kMaxRanks;
constexpr int XG_MAX_BLOCKS = edl_xgmi::kMaxBlocks;

struct XgmiPeers {
  char* data[XG_MAX_RANKS][2];     // peer p's data buffer for parity 0/1 (own rank included)
  uint32_t* flags[XG_MAX_RANKS];   // peer p's flag array [phase 2][src rank 8][block 256]
};

__device__ __forceinline__ uint32_t* flag_at(uint32_t* base, int phase, int src, int blk) {
  return base + (phase * XG_MAX_RANKS + src) * XG_MAX_BLOCKS + blk;
}

__device__ __forceinline__ uint64_t now_ticks() { return wall_clock64(); }  // constant 100 MHz

// Workgroup barrier with the same workgroup index on every rank, for `phase`.
// Returns false (for every thread of the workgroup) on abort or deadline.
__device__ bool xg_barrier(const XgmiPeers& P, int rank, int nranks, int phase, uint32_t round,
                           const volatile int* abort_word, uint64_t deadline, int* status) {
  __shared__ int ok;
  __syncthreads();  // this workgroup's writes are complete (workgroup scope)
  if (threadIdx.x == 0) {
    __threadfence_system();  // ... and written back past L2 for the peers
    for (int p = 0; p < nranks; ++p)
      __hip_atomic_store(flag_at(P.flags[p], phase, rank, blockIdx.x), round, __ATOMIC_RELEASE,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    int good = 1;
    uint32_t* mine = P.flags[rank];
    for (int p = 0; p < nranks && good; ++p) {
      uint32_t* f = flag_at(mine, phase, p, blockIdx.x);
      while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < round) {
        if (*abort_word || now_ticks() > deadline) {
          good = 0;
          __hip_atomic_store(status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);  // host-mapped word
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
    ok = good;
  }
  __syncthreads();
  return ok != 0;
}

enum XgOp { XG_SUM = 0, XG_MAX = 1 };

template <int OP>
__device__ __forceinline__ float xg_combine(float a, float b) {
  return OP == XG_SUM ? a + b : fmaxf(a, b);
}

template <typename T>
struct Vec;  // 16 B of T with f32 accumulation
template <>
struct Vec<float> {
  static constexpr int N = 4;
  template <int OP = XG_SUM>
  __device__ static void acc(float (&a)[8], const u32x4& v) {
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = xg_combine<OP>(a[i], __uint_as_float(v[i]));
  }
  __device__ static u32x4 pack(const float (&a)[8]) {
    return u32x4{__float_as_uint(a[0]), __float_as_uint(a[1]), __float_as_uint(a[2]), __float_as_uint(a[3])};
  }
};
template <>
struct Vec<bf16_t> {
  static constexpr int N = 8;
  template <int OP = XG_SUM>
  __device__ static void acc(float (&a)[8], const u32x4& v) {
    float f[8];
    unpack8(v, f);
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = xg_combine<OP>(a[i], f[i]);
  }
  __device__ static u32x4 pack(const float (&a)[8]) { return pack8(a); }
};

// combine 16-byte vector i over all ranks' buffers (own rank first: local HBM)
template <typename T, int OP = XG_SUM>
__device__ __forceinline__ u32x4 sum_vec(const XgmiPeers& P, int par, int rank, int nranks, int64_t vi) {
  const float init = OP == XG_SUM ? 0.f : -INFINITY;
  float a[8] = {init, init, init, init, init, init, init, init};
  for (int k = 0; k < nranks; ++k) {
    const int p = (rank + k) % nranks;  // stagger peers so ranks do not all hit one link at once
    Vec<T>::template acc<OP>(a, reinterpret_cast<const u32x4*>(P.data[p][par])[vi]);
  }
  return Vec<T>::pack(a);
}

// One-shot all-reduce with MAX (vocab-parallel cross-entropy's row max); the SUM
// forms are the kernels below.
template <typename T>
__global__ __launch_bounds__(512) void xgmi_oneshot_max_kernel(XgmiPeers P, const T* __restrict__ in,
                                                               T* __restrict__ out, int64_t nvec, int rank,
                                                               int nranks, uint32_t round, const int* abort_word,
                                                               uint64_t timeout_ticks, int* status) {
  const int par = round & 1;
  const uint64_t deadline = now_ticks() + timeout_ticks;
  const int64_t per = (nvec + gridDim.x - 1) / gridDim.x;
  const int64_t lo = blockIdx.x * per, hi = min(nvec, lo + per);
  u32x4* mine = reinterpret_cast<u32x4*>(P.data[rank][par]);
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) mine[i] = reinterpret_cast<const u32x4*>(in)[i];
  if (!xg_barrier(P, rank, nranks, 0, round, abort_word, deadline, status)) return;
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x)
    reinterpret_cast<u32x4*>(out)[i] = sum_vec<T, XG_MAX>(P, par, rank, nranks, i);
}

// All-gather: every rank stages its nvec vectors, then copies rank p's into
// out[p * out_stride ...] straight from p's buffer (N-1 links in parallel).
__global__ __launch_bounds__(512) void xgmi_allgather_kernel(XgmiPeers P, const u32x4* __restrict__ in,
                                                             u32x4* __restrict__ out, int64_t nvec,
                                                             int64_t out_stride, int rank, int nranks, uint32_t round,
                                                             const int* abort_word, uint64_t timeout_ticks,
                                                             int* status) {
  const int par = round & 1;
  const uint64_t deadline = now_ticks() + timeout_ticks;
  const int64_t per = (nvec + gridDim.x - 1) / gridDim.x;
  const int64_t lo = blockIdx.x * per, hi = min(nvec, lo + per);
  u32x4* mine = reinterpret_cast<u32x4*>(P.data[rank][par]);
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) mine[i] = in[i];
  if (!xg_barrier(P, rank, nranks, 0, round, abort_word, deadline, status)) return;
  for (int k = 0; k < nranks; ++k) {
    const int p = (rank + k) % nranks;
    const u32x4* pb = reinterpret_cast<const u32x4*>(P.data[p][par]);
    for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) out[p * out_stride + i] = pb[i];
  }
}

// Reduce-scatter (SUM): every rank stages all nranks slices (slice p from
// in[p * in_stride ...]), then sums its own slice from every rank's buffer.
template <typename T>
__global__ __launch_bounds__(512) void xgmi_reducescatter_kernel(XgmiPeers P, const T* __restrict__ in,
                                                                 T* __restrict__ out, int64_t nvec, int64_t in_stride,
                                                                 int rank, int nranks, uint32_t round,
                                                                 const int* abort_word, uint64_t timeout_ticks,
                                                                 int* status) {
  const int par = round & 1;
  const uint64_t deadline = now_ticks() + timeout_ticks;
  const int64_t per = (nvec + gridDim.x - 1) / gridDim.x;
  const int64_t lo = blockIdx.x * per, hi = min(nvec, lo + per);
  u32x4* mine = reinterpret_cast<u32x4*>(P.data[rank][par]);
  const u32x4* src = reinterpret_cast<const u32x4*>(in);
  for (int p = 0; p < nranks; ++p)
    for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) mine[p * nvec + i] = src[p * in_stride + i];
  if (!xg_barrier(P, rank, nranks, 0, round, abort_word, deadline, status)) return;
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x)
    reinterpret_cast<u32x4*>(out)[i] = sum_vec<T>(P, par, rank, nranks, rank * nvec + i);
}

template <typename T>
__global__ __launch_bounds__(512) void xgmi_oneshot_kernel(XgmiPeers P, const T* __restrict__ in, T* __restrict__ out,
                                                           int64_t nvec, int rank, int nranks, uint32_t round,
                                                           const int* abort_word, uint64_t timeout_ticks,
                                                           int* status) {
  const int par = round & 1;
  const uint64_t deadline = now_ticks() + timeout_ticks;
  const int64_t per = (nvec + gridDim.x - 1) / gridDim.x;
  const int64_t lo = blockIdx.x * per, hi = min(nvec, lo + per);
  u32x4* mine = reinterpret_cast<u32x4*>(P.data[rank][par]);
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) mine[i] = reinterpret_cast<const u32x4*>(in)[i];
  if (!xg_barrier(P, rank, nranks, 0, round, abort_word, deadline, status)) return;
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x)
    reinterpret_cast<u32x4*>(out)[i] = sum_vec<T>(P, par, rank, nranks, i);
}

// Two-shot: vectors are split into nranks chunks; workgroup b owns the same
// sub-range of every chunk on every rank.
template <typename T>
__global__ __launch_bounds__(512) void xgmi_twoshot_kernel(XgmiPeers P, const T* __restrict__ in, T* __restrict__ out,
                                                           int64_t nvec, int rank, int nranks, uint32_t round,
                                                           const int* abort_word, uint64_t timeout_ticks,
                                                           int* status) {
  const int par = round & 1;
  const uint64_t deadline = now_ticks() + timeout_ticks;
  const int64_t chunk = (nvec + nranks - 1) / nranks;
  const int64_t per = (chunk + gridDim.x - 1) / gridDim.x;
  const int64_t lo = blockIdx.x * per, hi = min(chunk, lo + per);
  u32x4* mine = reinterpret_cast<u32x4*>(P.data[rank][par]);
  const u32x4* src = reinterpret_cast<const u32x4*>(in);
  // stage: my sub-range of every chunk
  for (int c = 0; c < nranks; ++c) {
    const int64_t base = c * chunk;
    for (int64_t i = lo + threadIdx.x; i < hi && base + i < nvec; i += blockDim.x) mine[base + i] = src[base + i];
  }
  if (!xg_barrier(P, rank, nranks, 0, round, abort_word, deadline, status)) return;
  // reduce-scatter: my chunk, summed from every rank, in place in my buffer
  {
    const int64_t base = rank * chunk;
    for (int64_t i = lo + threadIdx.x; i < hi && base + i < nvec; i += blockDim.x)
      mine[base + i] = sum_vec<T>(P, par, rank, nranks, base + i);
  }
  if (!xg_barrier(P, rank, nranks, 1, round, abort_word, deadline, status)) return;
  // all-gather: chunk p from rank p
  u32x4* dst = reinterpret_cast<u32x4*>(out);
  for (int k = 0; k < nranks; ++k) {
    const int p = (rank + k) % nranks;
    const int64_t base = p * chunk;
    const u32x4* pb = reinterpret_cast<const u32x4*>(P.data[p][par]);
    for (int64_t i = lo + threadIdx.x; i < hi && base + i < nvec; i += blockDim.x) dst[base + i] = pb[base + i];
  }
}

}  // namespace

extern "C" {

int edl_xgmi_max_ranks() { return XG_MAX_RANKS; }
int edl_xgmi_max_blocks() { return XG_MAX_BLOCKS; }
int edl_xgmi_flag_bytes() { return edl_xgmi::kFlagBytes; }

// data[r*2 + parity], flags[r] : device pointers valid in this process (own + mapped peers)
// dtype: 0 = fp32, 1 = bf16.  nbytes must be a multiple of 16 and fit the workspace.
// algo: 0 = one-shot, 1 = two-shot.  Returns 0 or a hipError; kernel-side
// failures (abort / timeout) are reported through *status (device int).
int edl_xgmi_allreduce(void* const* data, void* const* flags, int nranks, int rank, const void* in, void* out,
                       int64_t nbytes, int dtype, int algo, uint32_t round, int blocks, const int* abort_word,
                       double timeout_s, int* status, hipStream_t s) {
  if (nranks < 1 || nranks > XG_MAX_RANKS || rank < 0 || rank >= nranks || (nbytes & 15) || blocks < 1 ||
      blocks > XG_MAX_BLOCKS)
    return (int)hipErrorInvalidValue;
  XgmiPeers P{};
  for (int r = 0; r < nranks; ++r) {
    P.data[r][0] = (char*)data[2 * r];
    P.data[r][1] = (char*)data[2 * r + 1];
    P.flags[r] = (uint32_t*)flags[r];
  }
  const int64_t nvec = nbytes / 16;
  const uint64_t ticks = (uint64_t)(timeout_s * 1e8);
#define EDL_XG(KERNEL, T)                                                                                     \
  KERNEL<T><<<blocks, 512, 0, s>>>(P, (const T*)in, (T*)out, nvec, rank, nranks, round, abort_word, ticks, \
                                   status)
  if (algo == 0) {
    if (dtype == 0) EDL_XG(xgmi_oneshot_kernel, float); else EDL_XG(xgmi_oneshot_kernel, bf16_t);
  } else {
    if (dtype == 0) EDL_XG(xgmi_twoshot_kernel, float); else EDL_XG(xgmi_twoshot_kernel, bf16_t);
  }
#undef EDL_XG
  EDL_LAUNCH_CHECK();
  return 0;
}

// Other collectives on the same workspace (TP / SP traffic).  kind:
//   0 = all-reduce MAX (one-shot) in -> out, nvec_in vectors;
//   1 = all-gather: in nvec_in vectors -> out[p * stride + i];
//   2 = reduce-scatter SUM: in[p * stride + i] (p < nranks, i < nvec_in) -> out nvec_in vectors.
// Sizes are in 16-byte vectors; the caller splits messages to fit the workspace
// (kind 2 stages nranks * nvec_in vectors).
int edl_xgmi_collective(void* const* data, void* const* flags, int nranks, int rank, const void* in, void* out,
                        int64_t nvec_in, int64_t stride, int dtype, int kind, uint32_t round, int blocks,
                        const int* abort_word, double timeout_s, int* status, hipStream_t s) {
  if (nranks < 1 || nranks > XG_MAX_RANKS || rank < 0 || rank >= nranks || nvec_in < 0 || blocks < 1 ||
      blocks > XG_MAX_BLOCKS || kind < 0 || kind > 2)
    return (int)hipErrorInvalidValue;
  XgmiPeers P{};
  for (int r = 0; r < nranks; ++r) {
    P.data[r][0] = (char*)data[2 * r];
    P.data[r][1] = (char*)data[2 * r + 1];
    P.flags[r] = (uint32_t*)flags[r];
  }
  const uint64_t ticks = (uint64_t)(timeout_s * 1e8);
  if (kind == 0) {
    if (dtype == 0)
      xgmi_oneshot_max_kernel<float><<<blocks, 512, 0, s>>>(P, (const float*)in, (float*)out, nvec_in, rank, nranks,
                                                            round, abort_word, ticks, status);
    else
      xgmi_oneshot_max_kernel<bf16_t><<<blocks, 512, 0, s>>>(P, (const bf16_t*)in, (bf16_t*)out, nvec_in, rank,
                                                             nranks, round, abort_word, ticks, status);
  } else if (kind == 1) {
    xgmi_allgather_kernel<<<blocks, 512, 0, s>>>(P, (const u32x4*)in, (u32x4*)out, nvec_in, stride, rank, nranks,
                                                 round, abort_word, ticks, status);
  } else {
    if (dtype == 0)
      xgmi_reducescatter_kernel<float><<<blocks, 512, 0, s>>>(P, (const float*)in, (float*)out, nvec_in, stride,
                                                              rank, nranks, round, abort_word, ticks, status);
    else
      xgmi_reducescatter_kernel<bf16_t><<<blocks, 512, 0, s>>>(P, (const bf16_t*)in, (bf16_t*)out, nvec_in,
                                                               stride, rank, nranks, round, abort_word, ticks,
                                                               status);
  }
  EDL_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
