// Custom xGMI collectives for one MI355X node.
//
// A node's GPUs are fully connected point-to-point (7 xGMI links each), so
// instead of a ring every rank reads every peer directly, spreading a
// message over all links at once.  Peer memory is mapped with IPC
// (csrc/runtime/xgmi.cpp).  Two kinds of peer memory exist:
//   * the staging workspace: two data buffers per rank (round parity) —
//     used for arbitrary tensors (TP / SP activations, small messages);
//   * registered buffers: the flat gradient buffer of every rank is mapped
//     by every peer once per epoch, so the DDP bucket all-reduce reads the
//     peers' gradients IN PLACE (no staging copy):
//       entry barrier  -> every rank's bucket is final
//       reduce-scatter -> rank r sums chunk r from all ranks into its own buffer
//       barrier        -> every reduced chunk is final
//       all-gather     -> rank r copies chunk p from rank p
//       exit barrier   -> no peer still reads rank r's chunk (backward of the
//                         next step may overwrite it)
//     Each byte crosses a link twice in total, spread over all 7 links,
//     instead of 2(N-1)/N hops around one ring per channel.
// Synchronisation is per workgroup (workgroup b of every rank covers the same
// sub-range of every chunk), with system-scope release/acquire on flags that
// live in uncached memory.  Flags carry the round number (monotone).  Every
// spin is bounded: it gives up when a host-mapped abort word is set (the
// elastic watchdog) or when the deadline — counted from THIS barrier's entry,
// on the constant-rate wall clock whose rate the host queries — passes; the
// first give-up records round / phase / workgroup / missing peer / waited ms
// in a host-mapped status record, so a failure describes itself.
//
// Memory-level parallelism: the reduce loops load U 16-byte vectors from
// each of the NR ranks before combining (NR is a template parameter, so the
// peer loop unrolls and 2*NR..4*NR loads are in flight per thread).
#include "../include/xgmi_layout.h"
#include "common.h"

using namespace edl;

namespace {

constexpr int XG_MAX_RANKS = edl_xgmi::kMaxRanks;
constexpr int XG_MAX_BLOCKS = edl_xgmi::kMaxBlocks;
constexpr int XG_THREADS = 512;

struct XgSync {
  uint32_t* flags[XG_MAX_RANKS];  // rank p's flag array [phase][src rank][block] (own included)
  const int* abort_word;          // host-mapped, set by the watchdog
  int* status;                    // host-mapped status record (kStatusWords ints)
  uint64_t timeout_ticks;         // per barrier, wall-clock ticks
  uint64_t ticks_per_ms;
  uint32_t round;
  int rank;
};

struct XgBufs {
  char* p[XG_MAX_RANKS];  // rank q's region, as mapped in this process
};

__device__ __forceinline__ uint32_t* flag_at(uint32_t* base, int phase, int src, int blk) {
  return base + (phase * XG_MAX_RANKS + src) * XG_MAX_BLOCKS + blk;
}

__device__ __forceinline__ uint64_t now_ticks() { return wall_clock64(); }

__device__ void xg_record(const XgSync& S, int phase, int peer, uint32_t seen, uint64_t waited, int reason) {
  int* st = S.status;
  const int vals[7] = {(int)S.round, phase, (int)blockIdx.x, peer, (int)seen,
                       (int)(waited / (S.ticks_per_ms ? S.ticks_per_ms : 1)), reason};
  for (int i = 0; i < 7; ++i) __hip_atomic_store(st + 1 + i, vals[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(st, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Workgroup barrier with the same workgroup index on every rank, for `phase`.
// Returns false (for every thread of the workgroup) on abort or deadline.
template <int NR>
__device__ bool xg_barrier(const XgSync& S, int phase) {
  __shared__ int ok;
  __syncthreads();  // this workgroup's writes are issued (workgroup scope)
  if (threadIdx.x == 0) {
    __threadfence_system();  // ... and visible past the L2 to the peers
#pragma unroll
    for (int p = 0; p < NR; ++p)
      __hip_atomic_store(flag_at(S.flags[p], phase, S.rank, blockIdx.x), S.round, __ATOMIC_RELEASE,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    int good = 1;
    const uint64_t t0 = now_ticks();
    for (int k = 1; k < NR && good; ++k) {
      int p = S.rank + k;
      p -= p >= NR ? NR : 0;
      uint32_t* f = flag_at(S.flags[S.rank], phase, p, blockIdx.x);
      uint32_t v;
      while ((v = __hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM)) < S.round) {
        const uint64_t waited = now_ticks() - t0;
        const int reason = *(volatile const int*)S.abort_word ? 1 : (waited > S.timeout_ticks ? 2 : 0);
        if (reason) {
          xg_record(S, phase, p, v, waited, reason);
          good = 0;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    // own flag (k = 0) needs no wait; an acquire still orders our later reads
    (void)__hip_atomic_load(flag_at(S.flags[S.rank], phase, S.rank, blockIdx.x), __ATOMIC_ACQUIRE,
                            __HIP_MEMORY_SCOPE_SYSTEM);
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
  template <int OP>
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
  template <int OP>
  __device__ static void acc(float (&a)[8], const u32x4& v) {
    float f[8];
    unpack8(v, f);
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = xg_combine<OP>(a[i], f[i]);
  }
  __device__ static u32x4 pack(const float (&a)[8]) { return pack8(a); }
};

template <int NR>
struct Unroll {
  static constexpr int U = NR <= 2 ? 4 : 2;  // 16-byte vectors per rank in flight per thread
};

// dst[i] = OP over q of src_q[i] for i in [lo, hi) (vector indices relative to
// the given pointers).  Own rank is read first (local HBM), peers staggered so
// ranks do not all hit one link at the same moment.
template <typename T, int NR, int OP>
__device__ __forceinline__ void reduce_range(const char* const (&src)[XG_MAX_RANKS], int rank, u32x4* dst, int64_t lo,
                                             int64_t hi) {
  constexpr int U = Unroll<NR>::U;
  const float init = OP == XG_SUM ? 0.f : -INFINITY;
  for (int64_t i0 = lo + threadIdx.x; i0 < hi; i0 += (int64_t)U * XG_THREADS) {
    u32x4 v[U][NR];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + (int64_t)u * XG_THREADS;
      if (i < hi) {
#pragma unroll
        for (int k = 0; k < NR; ++k) {
          int q = rank + k;
          q -= q >= NR ? NR : 0;
          v[u][k] = reinterpret_cast<const u32x4*>(src[q])[i];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + (int64_t)u * XG_THREADS;
      if (i < hi) {
        float a[8] = {init, init, init, init, init, init, init, init};
#pragma unroll
        for (int k = 0; k < NR; ++k) Vec<T>::template acc<OP>(a, v[u][k]);
        dst[i] = Vec<T>::pack(a);
      }
    }
  }
}

// dst[p * chunk + i] = src_p[p * chunk + i] for every rank p (skip own when
// skip_own), i in [lo, hi), p * chunk + i < nvec.
template <int NR>
__device__ __forceinline__ void gather_range(const char* const (&src)[XG_MAX_RANKS], int rank, u32x4* dst,
                                             int64_t chunk, int64_t nvec, int64_t lo, int64_t hi, bool skip_own) {
  constexpr int U = Unroll<NR>::U;
  for (int64_t i0 = lo + threadIdx.x; i0 < hi; i0 += (int64_t)U * XG_THREADS) {
    u32x4 v[U][NR];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + (int64_t)u * XG_THREADS;
#pragma unroll
      for (int k = 0; k < NR; ++k) {
        int p = rank + k;
        p -= p >= NR ? NR : 0;
        const int64_t j = p * chunk + i;
        if (i < hi && j < nvec && !(skip_own && k == 0)) v[u][k] = reinterpret_cast<const u32x4*>(src[p])[j];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + (int64_t)u * XG_THREADS;
#pragma unroll
      for (int k = 0; k < NR; ++k) {
        int p = rank + k;
        p -= p >= NR ? NR : 0;
        const int64_t j = p * chunk + i;
        if (i < hi && j < nvec && !(skip_own && k == 0)) dst[j] = v[u][k];
      }
    }
  }
}

__device__ __forceinline__ void copy_range(const u32x4* __restrict__ src, u32x4* __restrict__ dst, int64_t lo,
                                           int64_t hi) {
  for (int64_t i = lo + threadIdx.x; i < hi; i += XG_THREADS) dst[i] = src[i];
}

__device__ __forceinline__ void block_range(int64_t n, int64_t& lo, int64_t& hi) {
  const int64_t per = (n + gridDim.x - 1) / gridDim.x;
  lo = blockIdx.x * per;
  hi = min(n, lo + per);
}

template <int NR>
__device__ __forceinline__ void offset_all(const XgBufs& B, int64_t vec_off, const char* (&out)[XG_MAX_RANKS]) {
#pragma unroll
  for (int q = 0; q < NR; ++q) out[q] = B.p[q] + vec_off * 16;
}

// ---- staged collectives (workspace buffers W, parity chosen by the host) -------------

// One-shot all-reduce (SUM or MAX): stage, barrier, combine all ranks' stages.
template <typename T, int NR, int OP>
__global__ __launch_bounds__(XG_THREADS) void xg_oneshot(XgSync S, XgBufs W, const u32x4* __restrict__ in,
                                                         u32x4* __restrict__ out, int64_t nvec) {
  int64_t lo, hi;
  block_range(nvec, lo, hi);
  copy_range(in, reinterpret_cast<u32x4*>(W.p[S.rank]), lo, hi);
  if (!xg_barrier<NR>(S, 0)) return;
  const char* src[XG_MAX_RANKS];
  offset_all<NR>(W, 0, src);
  reduce_range<T, NR, OP>(src, S.rank, out, lo, hi);
}

// Two-shot all-reduce of an arbitrary tensor through the workspace.
template <typename T, int NR>
__global__ __launch_bounds__(XG_THREADS) void xg_twoshot_staged(XgSync S, XgBufs W, const u32x4* __restrict__ in,
                                                                u32x4* __restrict__ out, int64_t nvec) {
  const int64_t chunk = (nvec + NR - 1) / NR;
  int64_t lo, hi;
  block_range(chunk, lo, hi);
  u32x4* mine = reinterpret_cast<u32x4*>(W.p[S.rank]);
  for (int c = 0; c < NR; ++c) {
    const int64_t base = c * chunk;
    copy_range(in + base, mine + base, lo, min(hi, nvec - base));
  }
  if (!xg_barrier<NR>(S, 0)) return;
  {
    const char* src[XG_MAX_RANKS];
    offset_all<NR>(W, S.rank * chunk, src);
    reduce_range<T, NR, XG_SUM>(src, S.rank, mine + S.rank * chunk, lo, min(hi, nvec - S.rank * chunk));
  }
  if (!xg_barrier<NR>(S, 1)) return;
  const char* src[XG_MAX_RANKS];
  offset_all<NR>(W, 0, src);
  gather_range<NR>(src, S.rank, out, chunk, nvec, lo, hi, false);
}

// All-gather: stage nvec vectors, then out[p * out_stride + i] from rank p's stage.
template <int NR>
__global__ __launch_bounds__(XG_THREADS) void xg_allgather(XgSync S, XgBufs W, const u32x4* __restrict__ in,
                                                           u32x4* __restrict__ out, int64_t nvec, int64_t out_stride) {
  int64_t lo, hi;
  block_range(nvec, lo, hi);
  copy_range(in, reinterpret_cast<u32x4*>(W.p[S.rank]), lo, hi);
  if (!xg_barrier<NR>(S, 0)) return;
  constexpr int U = Unroll<NR>::U;
  for (int64_t i0 = lo + threadIdx.x; i0 < hi; i0 += (int64_t)U * XG_THREADS) {
    u32x4 v[U][NR];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + (int64_t)u * XG_THREADS;
#pragma unroll
      for (int k = 0; k < NR; ++k) {
        int p = S.rank + k;
        p -= p >= NR ? NR : 0;
        if (i < hi) v[u][k] = reinterpret_cast<const u32x4*>(W.p[p])[i];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + (int64_t)u * XG_THREADS;
#pragma unroll
      for (int k = 0; k < NR; ++k) {
        int p = S.rank + k;
        p -= p >= NR ? NR : 0;
        if (i < hi) out[p * out_stride + i] = v[u][k];
      }
    }
  }
}

// Reduce-scatter (SUM): stage all NR slices (slice p from in[p * in_stride ...]),
// then sum this rank's slice from every rank's stage.
template <typename T, int NR>
__global__ __launch_bounds__(XG_THREADS) void xg_reducescatter(XgSync S, XgBufs W, const u32x4* __restrict__ in,
                                                               u32x4* __restrict__ out, int64_t nvec,
                                                               int64_t in_stride) {
  int64_t lo, hi;
  block_range(nvec, lo, hi);
  u32x4* mine = reinterpret_cast<u32x4*>(W.p[S.rank]);
  for (int p = 0; p < NR; ++p) copy_range(in + p * in_stride, mine + p * nvec, lo, hi);
  if (!xg_barrier<NR>(S, 0)) return;
  const char* src[XG_MAX_RANKS];
  offset_all<NR>(W, S.rank * nvec, src);
  reduce_range<T, NR, XG_SUM>(src, S.rank, out, lo, hi);
}

// ---- in-place two-shot on registered buffers (DDP gradient buckets) -------------------

template <typename T, int NR>
__global__ __launch_bounds__(XG_THREADS) void xg_twoshot_inplace(XgSync S, XgBufs G, int64_t nvec) {
  const int64_t chunk = (nvec + NR - 1) / NR;
  int64_t lo, hi;
  block_range(chunk, lo, hi);
  u32x4* mine = reinterpret_cast<u32x4*>(G.p[S.rank]);
  if (!xg_barrier<NR>(S, 0)) return;  // every rank's bucket is final
  {
    const char* src[XG_MAX_RANKS];
    offset_all<NR>(G, S.rank * chunk, src);
    reduce_range<T, NR, XG_SUM>(src, S.rank, mine + S.rank * chunk, lo, min(hi, nvec - S.rank * chunk));
  }
  if (!xg_barrier<NR>(S, 1)) return;  // every reduced chunk is final
  {
    const char* src[XG_MAX_RANKS];
    offset_all<NR>(G, 0, src);
    gather_range<NR>(src, S.rank, mine, chunk, nvec, lo, hi, true);
  }
  xg_barrier<NR>(S, 2);  // nobody still reads my chunk
}

// Multi-source pull (state transfer to joiners / replacements): every rank NOT in
// holder_mask copies the message from the holders, slice k from the k-th holder,
// so a receiver's inbound traffic is spread over one xGMI link per holder.
// Workgroup b serves holder (b mod nh); the holders' workgroups only take part
// in the entry barrier (their copy is final) and the exit barrier (nobody still
// reads it), so they may train on right after.
template <int NR>
__global__ __launch_bounds__(XG_THREADS) void xg_pull(XgSync S, XgBufs G, int64_t nvec, uint32_t holder_mask) {
  if (!xg_barrier<NR>(S, 0)) return;
  if (!((holder_mask >> S.rank) & 1u)) {
    int hs[XG_MAX_RANKS];
    int nh = 0;
#pragma unroll
    for (int p = 0; p < NR; ++p)
      if ((holder_mask >> p) & 1u) hs[nh++] = p;
    if (nh > 0) {
      const int k = blockIdx.x % nh;
      const int nb = (gridDim.x - k + nh - 1) / nh;  // workgroups serving holder k
      const int bi = blockIdx.x / nh;
      const int64_t slice = (nvec + nh - 1) / nh;
      const int64_t s0 = k * slice, s1 = min(nvec, s0 + slice);
      const int64_t per = (s1 - s0 + nb - 1) / nb;
      const int64_t lo = s0 + bi * per, hi = min(s1, lo + per);
      const u32x4* src = reinterpret_cast<const u32x4*>(G.p[hs[k]]);
      u32x4* dst = reinterpret_cast<u32x4*>(G.p[S.rank]);
      constexpr int U = 8;
      for (int64_t i0 = lo + threadIdx.x; i0 < hi; i0 += (int64_t)U * XG_THREADS) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int64_t i = i0 + (int64_t)u * XG_THREADS;
          if (i < hi) v[u] = src[i];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int64_t i = i0 + (int64_t)u * XG_THREADS;
          if (i < hi) dst[i] = v[u];
        }
      }
    }
  }
  xg_barrier<NR>(S, 2);
}

// Staged multi-source pull for tensors too large to map (one window per launch): the
// k-th holder stages slice k of the window into its workspace buffer, every receiver
// copies slice k from holder k's workspace.  Round parity protects the buffers as in
// the staged all-reduce; workgroup b of a receiver reads only what workgroup b of each
// holder staged.  src: this rank's tensor (holders), dst: the same tensor
// (receivers); win_off / win_len in 16-byte vectors.
template <int NR>
__global__ __launch_bounds__(XG_THREADS) void xg_pull_staged(XgSync S, XgBufs W, const u32x4* __restrict__ src,
                                                             u32x4* __restrict__ dst, int64_t win_off,
                                                             int64_t win_len, uint32_t holder_mask) {
  int hs[XG_MAX_RANKS];
  int nh = 0, me = -1;
#pragma unroll
  for (int p = 0; p < NR; ++p)
    if ((holder_mask >> p) & 1u) {
      if (p == S.rank) me = nh;
      hs[nh++] = p;
    }
  const int64_t slice = (win_len + nh - 1) / nh;
  if (me >= 0) {   // holder: stage my slice of the window
    const int64_t s0 = (int64_t)me * slice, n = min(slice, win_len - s0);
    int64_t lo, hi;
    block_range(n, lo, hi);
    copy_range(src + win_off + s0, reinterpret_cast<u32x4*>(W.p[S.rank]), lo, hi);
  }
  if (!xg_barrier<NR>(S, 0)) return;
  if (me < 0) {
    // receiver: workgroup b copies, from EVERY holder k, exactly the sub-range holder k's
    // workgroup b staged (the barrier above only orders workgroup b against workgroup b)
    constexpr int U = 4;
    for (int k = 0; k < nh; ++k) {
      const int64_t s0 = (int64_t)k * slice, n = max<int64_t>(0, min(slice, win_len - s0));
      int64_t lo, hi;
      block_range(n, lo, hi);
      const u32x4* from = reinterpret_cast<const u32x4*>(W.p[hs[k]]);
      u32x4* to = dst + win_off + s0;
      for (int64_t i0 = lo + threadIdx.x; i0 < hi; i0 += (int64_t)U * XG_THREADS) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int64_t i = i0 + (int64_t)u * XG_THREADS;
          if (i < hi) v[u] = from[i];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int64_t i = i0 + (int64_t)u * XG_THREADS;
          if (i < hi) to[i] = v[u];
        }
      }
    }
  }
}

// Flag-only barrier across ranks (e.g. before buffers are re-registered or freed).
template <int NR>
__global__ __launch_bounds__(64) void xg_barrier_kernel(XgSync S) {
  xg_barrier<NR>(S, 0);
}

// ---- host helpers ------------------------------------------------------------------

uint64_t ticks_per_s() {
  static uint64_t cached[64] = {0};
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= 64) dev = 0;
  if (!cached[dev]) {
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0) khz = 100000;
    cached[dev] = (uint64_t)khz * 1000ull;
  }
  return cached[dev];
}

XgSync make_sync(void* const* flags, int nranks, int rank, uint32_t round, const int* abort_word, double timeout_s,
                 int* status) {
  XgSync S{};
  for (int r = 0; r < nranks; ++r) S.flags[r] = (uint32_t*)flags[r];
  S.abort_word = abort_word;
  S.status = status;
  const uint64_t hz = ticks_per_s();
  S.ticks_per_ms = hz / 1000;
  S.timeout_ticks = (uint64_t)(timeout_s * (double)hz);
  S.round = round;
  S.rank = rank;
  return S;
}

XgBufs parity_bufs(void* const* data, int nranks, int par) {
  XgBufs W{};
  for (int r = 0; r < nranks; ++r) W.p[r] = (char*)data[2 * r + par];
  return W;
}

bool bad_common(int nranks, int rank, int blocks) {
  return nranks < 1 || nranks > XG_MAX_RANKS || rank < 0 || rank >= nranks || blocks < 1 || blocks > XG_MAX_BLOCKS;
}

#define XG_DISPATCH_NR(NRV, BODY)          \
  switch (NRV) {                           \
    case 1: { constexpr int NR = 1; BODY; } break; \
    case 2: { constexpr int NR = 2; BODY; } break; \
    case 3: { constexpr int NR = 3; BODY; } break; \
    case 4: { constexpr int NR = 4; BODY; } break; \
    case 5: { constexpr int NR = 5; BODY; } break; \
    case 6: { constexpr int NR = 6; BODY; } break; \
    case 7: { constexpr int NR = 7; BODY; } break; \
    default: { constexpr int NR = 8; BODY; } break; \
  }

}  // namespace

extern "C" {

int edl_xgmi_max_ranks() { return XG_MAX_RANKS; }
int edl_xgmi_max_blocks() { return XG_MAX_BLOCKS; }
int edl_xgmi_flag_bytes() { return edl_xgmi::kFlagBytes; }
int64_t edl_xgmi_wallclock_hz() { return (int64_t)ticks_per_s(); }

// Staged all-reduce.  data[r*2 + parity], flags[r]: device pointers valid in this
// process (own + mapped peers).  dtype: 0 = fp32, 1 = bf16.  nbytes must be a
// multiple of 16 and fit one workspace buffer.  algo: 0 = one-shot, 1 = two-shot.
// Returns 0 or a hipError; kernel-side give-ups (abort / deadline) are reported
// through the status record.
int edl_xgmi_allreduce(void* const* data, void* const* flags, int nranks, int rank, const void* in, void* out,
                       int64_t nbytes, int dtype, int algo, uint32_t round, int blocks, const int* abort_word,
                       double timeout_s, int* status, hipStream_t s) {
  if (bad_common(nranks, rank, blocks) || (nbytes & 15)) return (int)hipErrorInvalidValue;
  const XgSync S = make_sync(flags, nranks, rank, round, abort_word, timeout_s, status);
  const XgBufs W = parity_bufs(data, nranks, round & 1);
  const int64_t nvec = nbytes / 16;
  const u32x4* i = (const u32x4*)in;
  u32x4* o = (u32x4*)out;
  if (algo == 0) {
    if (dtype == 0) {
      XG_DISPATCH_NR(nranks, (xg_oneshot<float, NR, XG_SUM><<<blocks, XG_THREADS, 0, s>>>(S, W, i, o, nvec)));
    } else {
      XG_DISPATCH_NR(nranks, (xg_oneshot<bf16_t, NR, XG_SUM><<<blocks, XG_THREADS, 0, s>>>(S, W, i, o, nvec)));
    }
  } else {
    if (dtype == 0) {
      XG_DISPATCH_NR(nranks, (xg_twoshot_staged<float, NR><<<blocks, XG_THREADS, 0, s>>>(S, W, i, o, nvec)));
    } else {
      XG_DISPATCH_NR(nranks, (xg_twoshot_staged<bf16_t, NR><<<blocks, XG_THREADS, 0, s>>>(S, W, i, o, nvec)));
    }
  }
  EDL_LAUNCH_CHECK();
  return 0;
}

// In-place two-shot SUM over registered buffers: bufs[r] = rank r's copy of the
// message (e.g. a gradient bucket), as mapped in this process; one launch for
// any size.  nbytes must be a multiple of 16.
int edl_xgmi_allreduce_inplace(void* const* bufs, void* const* flags, int nranks, int rank, int64_t nbytes, int dtype,
                               uint32_t round, int blocks, const int* abort_word, double timeout_s, int* status,
                               hipStream_t s) {
  if (bad_common(nranks, rank, blocks) || (nbytes & 15)) return (int)hipErrorInvalidValue;
  const XgSync S = make_sync(flags, nranks, rank, round, abort_word, timeout_s, status);
  XgBufs G{};
  for (int r = 0; r < nranks; ++r) G.p[r] = (char*)bufs[r];
  const int64_t nvec = nbytes / 16;
  if (dtype == 0) {
    XG_DISPATCH_NR(nranks, (xg_twoshot_inplace<float, NR><<<blocks, XG_THREADS, 0, s>>>(S, G, nvec)));
  } else {
    XG_DISPATCH_NR(nranks, (xg_twoshot_inplace<bf16_t, NR><<<blocks, XG_THREADS, 0, s>>>(S, G, nvec)));
  }
  EDL_LAUNCH_CHECK();
  return 0;
}

// Multi-source pull over registered buffers (see xg_pull): bufs[r] = rank r's copy.
int edl_xgmi_pull(void* const* bufs, void* const* flags, int nranks, int rank, int64_t nbytes, uint32_t holder_mask,
                  uint32_t round, int blocks, const int* abort_word, double timeout_s, int* status, hipStream_t s) {
  if (bad_common(nranks, rank, blocks) || (nbytes & 15) || holder_mask == 0 || (holder_mask >> nranks))
    return (int)hipErrorInvalidValue;
  const XgSync S = make_sync(flags, nranks, rank, round, abort_word, timeout_s, status);
  XgBufs G{};
  for (int r = 0; r < nranks; ++r) G.p[r] = (char*)bufs[r];
  XG_DISPATCH_NR(nranks, (xg_pull<NR><<<blocks, XG_THREADS, 0, s>>>(S, G, nbytes / 16, holder_mask)));
  EDL_LAUNCH_CHECK();
  return 0;
}

// Staged multi-source pull of one window (see xg_pull_staged); the holders' slices of
// the window (win_bytes / #holders each) must fit one workspace buffer.
int edl_xgmi_pull_staged(void* const* data, void* const* flags, int nranks, int rank, const void* src, void* dst,
                         int64_t win_off_bytes, int64_t win_bytes, uint32_t holder_mask, uint32_t round, int blocks,
                         const int* abort_word, double timeout_s, int* status, hipStream_t s) {
  if (bad_common(nranks, rank, blocks) || (win_off_bytes & 15) || (win_bytes & 15) || holder_mask == 0 ||
      (holder_mask >> nranks))
    return (int)hipErrorInvalidValue;
  const XgSync S = make_sync(flags, nranks, rank, round, abort_word, timeout_s, status);
  const XgBufs W = parity_bufs(data, nranks, round & 1);
  XG_DISPATCH_NR(nranks, (xg_pull_staged<NR><<<blocks, XG_THREADS, 0, s>>>(S, W, (const u32x4*)src, (u32x4*)dst,
                                                                            win_off_bytes / 16, win_bytes / 16,
                                                                            holder_mask)));
  EDL_LAUNCH_CHECK();
  return 0;
}

// Barrier on the flags only (one workgroup per rank).
int edl_xgmi_barrier(void* const* flags, int nranks, int rank, uint32_t round, const int* abort_word,
                     double timeout_s, int* status, hipStream_t s) {
  if (bad_common(nranks, rank, 1)) return (int)hipErrorInvalidValue;
  const XgSync S = make_sync(flags, nranks, rank, round, abort_word, timeout_s, status);
  XG_DISPATCH_NR(nranks, (xg_barrier_kernel<NR><<<1, 64, 0, s>>>(S)));
  EDL_LAUNCH_CHECK();
  return 0;
}

// Other staged collectives (TP / SP traffic).  kind:
//   0 = all-reduce MAX (one-shot) in -> out, nvec_in vectors;
//   1 = all-gather: in nvec_in vectors -> out[p * stride + i];
//   2 = reduce-scatter SUM: in[p * stride + i] (p < nranks, i < nvec_in) -> out nvec_in vectors.
// Sizes are in 16-byte vectors; the caller splits messages to fit the workspace
// (kind 2 stages nranks * nvec_in vectors).
int edl_xgmi_collective(void* const* data, void* const* flags, int nranks, int rank, const void* in, void* out,
                        int64_t nvec_in, int64_t stride, int dtype, int kind, uint32_t round, int blocks,
                        const int* abort_word, double timeout_s, int* status, hipStream_t s) {
  if (bad_common(nranks, rank, blocks) || nvec_in < 0 || kind < 0 || kind > 2) return (int)hipErrorInvalidValue;
  const XgSync S = make_sync(flags, nranks, rank, round, abort_word, timeout_s, status);
  const XgBufs W = parity_bufs(data, nranks, round & 1);
  const u32x4* i = (const u32x4*)in;
  u32x4* o = (u32x4*)out;
  if (kind == 0) {
    if (dtype == 0) {
      XG_DISPATCH_NR(nranks, (xg_oneshot<float, NR, XG_MAX><<<blocks, XG_THREADS, 0, s>>>(S, W, i, o, nvec_in)));
    } else {
      XG_DISPATCH_NR(nranks, (xg_oneshot<bf16_t, NR, XG_MAX><<<blocks, XG_THREADS, 0, s>>>(S, W, i, o, nvec_in)));
    }
  } else if (kind == 1) {
    XG_DISPATCH_NR(nranks, (xg_allgather<NR><<<blocks, XG_THREADS, 0, s>>>(S, W, i, o, nvec_in, stride)));
  } else {
    if (dtype == 0) {
      XG_DISPATCH_NR(nranks,
                     (xg_reducescatter<float, NR><<<blocks, XG_THREADS, 0, s>>>(S, W, i, o, nvec_in, stride)));
    } else {
      XG_DISPATCH_NR(nranks,
                     (xg_reducescatter<bf16_t, NR><<<blocks, XG_THREADS, 0, s>>>(S, W, i, o, nvec_in, stride)));
    }
  }
  EDL_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
