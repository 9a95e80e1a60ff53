// Parameter-server data-plane kernels.
//
// Embedding tables of CTR-style models (the reference's example job is
// "elastic-deepctr-job", docs/design/elastic-training-operator.md:35) live on
// the PS as fp32 [rows, dim].  Workers touch a few thousand rows per step, so
// push/pull are row-sparse:
//   * pull  = gather rows (edl_embed_gather): one 64-lane wave per row, 16-B
//     loads; the table pointer may be an IPC-mapped peer pointer, then the
//     rows stream over xGMI straight into the worker's HBM (bf16 or fp32 out);
//   * push  = segment-sum of duplicate ids into a compact [unique, dim]
//     gradient (edl_embed_scatter_add: fp32 atomics into an L2-resident
//     buffer), then a lazy AdamW/Adagrad/SGD on exactly the touched rows
//     (edl_sparse_adamw_rows) — untouched rows keep their moments, as in
//     TF's lazy Adam, so the cost is O(touched rows), not O(table);
//   * dense pull with cast (edl_ps_pull_cast): fp32 PS shard -> bf16 worker
//     params, reading a peer pointer over xGMI;
//   * multi-tensor dense push / pull (edl_ps_multi_copy): ONE launch moves every
//     parameter of a shard between the worker's (scattered, bf16 or fp32)
//     tensors and the PS's flat fp32 buffer — push writes gradients, cast to
//     fp32, straight into the PS's inbox (peer writes over xGMI), pull reads
//     the fp32 shard and writes the worker's parameters.  A tensor table in
//     device memory drives it; workgroup -> (tensor, chunk) by a binary search
//     over the per-tensor block prefix.
// Index validity is checked on the host side of every entry (rows bound); a
// bad id is clamped to a zero row on gather and dropped on scatter instead of
// faulting the device.
#include "common.h"

using namespace edl;

namespace {

constexpr int kRowBlock = 256;  // 4 waves, one row per wave

// dim % 4 == 0; one wave per row, each lane moves 4 floats per iteration.
template <bool OUT_BF16>
__global__ __launch_bounds__(kRowBlock) void embed_gather_kernel(const float* __restrict__ table,
                                                                 const int64_t* __restrict__ idx, int64_t n, int dim,
                                                                 int64_t rows, void* __restrict__ out) {
  const int64_t r = (int64_t)blockIdx.x * (kRowBlock / kWave) + (threadIdx.x >> 6);
  if (r >= n) return;
  const int lane = threadIdx.x & 63;
  const int64_t id = idx[r];
  const bool ok = id >= 0 && id < rows;
  const f32x4* src = reinterpret_cast<const f32x4*>(table + (ok ? id : 0) * (int64_t)dim);
  const int d4 = dim >> 2;
  for (int c = lane; c < d4; c += kWave) {
    f32x4 v = ok ? src[c] : f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (OUT_BF16) {
      u32x2 o{pack2(v[0], v[1]), pack2(v[2], v[3])};
      reinterpret_cast<u32x2*>(static_cast<bf16_t*>(out) + r * (int64_t)dim)[c] = o;
    } else {
      reinterpret_cast<f32x4*>(static_cast<float*>(out) + r * (int64_t)dim)[c] = v;
    }
  }
}

template <bool IN_BF16>
__global__ __launch_bounds__(kRowBlock) void embed_scatter_add_kernel(float* __restrict__ acc,
                                                                      const int64_t* __restrict__ idx,
                                                                      const void* __restrict__ grad, int64_t n,
                                                                      int dim, int64_t rows) {
  const int64_t r = (int64_t)blockIdx.x * (kRowBlock / kWave) + (threadIdx.x >> 6);
  if (r >= n) return;
  const int64_t id = idx[r];
  if (id < 0 || id >= rows) return;
  const int lane = threadIdx.x & 63;
  float* dst = acc + id * (int64_t)dim;
  const int d4 = dim >> 2;
  for (int c = lane; c < d4; c += kWave) {
    float g[4];
    if constexpr (IN_BF16) {
      u32x2 w = reinterpret_cast<const u32x2*>(static_cast<const bf16_t*>(grad) + r * (int64_t)dim)[c];
      g[0] = bflo(w[0]); g[1] = bfhi(w[0]); g[2] = bflo(w[1]); g[3] = bfhi(w[1]);
    } else {
      f32x4 w = reinterpret_cast<const f32x4*>(static_cast<const float*>(grad) + r * (int64_t)dim)[c];
      g[0] = w[0]; g[1] = w[1]; g[2] = w[2]; g[3] = w[3];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) unsafeAtomicAdd(dst + 4 * c + j, g[j]);
  }
}

struct SparseOpt {
  int kind;  // 0 = AdamW, 1 = Adagrad, 2 = SGD
  float lr, beta1, beta2, eps, wd, step_size, inv_bc2_sqrt, scale;
};

// one wave updates table row `id` with gradient row G (lazy AdamW / Adagrad / SGD)
__device__ __forceinline__ void update_row(float* __restrict__ w, float* __restrict__ m, float* __restrict__ v,
                                           int64_t id, const float* __restrict__ grow, int dim, const SparseOpt& o,
                                           int lane);

// Update table rows rows[u] with compact gradient grad[u, :].
__global__ __launch_bounds__(kRowBlock) void sparse_rows_update_kernel(float* __restrict__ w, float* __restrict__ m,
                                                                       float* __restrict__ v,
                                                                       const int64_t* __restrict__ rows_idx,
                                                                       const float* __restrict__ grad, int64_t nu,
                                                                       int dim, int64_t rows, SparseOpt o) {
  const int64_t u = (int64_t)blockIdx.x * (kRowBlock / kWave) + (threadIdx.x >> 6);
  if (u >= nu) return;
  const int64_t id = rows_idx[u];
  if (id < 0 || id >= rows) return;
  update_row(w, m, v, id, grad + u * (int64_t)dim, dim, o, threadIdx.x & 63);
}

// PS side of the GPU sparse push: the rows a worker wrote into its inbox (local row ids,
// fp32 gradients, the row count written last by the worker's count kernel).  The count is
// read on the device (no host round trip); a grid-stride loop covers it.
__global__ __launch_bounds__(kRowBlock) void sparse_inbox_update_kernel(float* __restrict__ w, float* __restrict__ m,
                                                                        float* __restrict__ v,
                                                                        const int64_t* __restrict__ ids,
                                                                        const float* __restrict__ grad,
                                                                        const int* __restrict__ count, int64_t cap,
                                                                        int dim, int64_t rows, SparseOpt o) {
  const int64_t n = min((int64_t)*count, cap);
  const int64_t nw = (int64_t)gridDim.x * (kRowBlock / kWave);
  for (int64_t u = (int64_t)blockIdx.x * (kRowBlock / kWave) + (threadIdx.x >> 6); u < n; u += nw) {
    const int64_t id = ids[u];
    if (id < 0 || id >= rows) continue;
    update_row(w, m, v, id, grad + u * (int64_t)dim, dim, o, threadIdx.x & 63);
  }
}

__device__ __forceinline__ void update_row(float* __restrict__ w, float* __restrict__ m, float* __restrict__ v,
                                           int64_t id, const float* __restrict__ grow, int dim, const SparseOpt& o,
                                           int lane) {
  const int d4 = dim >> 2;
  f32x4* W = reinterpret_cast<f32x4*>(w + id * (int64_t)dim);
  f32x4* M = m ? reinterpret_cast<f32x4*>(m + id * (int64_t)dim) : nullptr;
  f32x4* V = v ? reinterpret_cast<f32x4*>(v + id * (int64_t)dim) : nullptr;
  const f32x4* G = reinterpret_cast<const f32x4*>(grow);
  const float decay = 1.f - o.lr * o.wd;
  for (int c = lane; c < d4; c += kWave) {
    f32x4 g = G[c] * o.scale, p = W[c];
    if (o.kind == 0) {
      f32x4 mm = M[c], vv = V[c];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        mm[j] = o.beta1 * mm[j] + (1.f - o.beta1) * g[j];
        vv[j] = o.beta2 * vv[j] + (1.f - o.beta2) * g[j] * g[j];
        p[j] = p[j] * decay - o.step_size * mm[j] / (sqrtf(vv[j]) * o.inv_bc2_sqrt + o.eps);
      }
      M[c] = mm;
      V[c] = vv;
    } else if (o.kind == 1) {
      f32x4 vv = V[c];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        vv[j] += g[j] * g[j];
        p[j] = p[j] * decay - o.lr * g[j] / (sqrtf(vv[j]) + o.eps);
      }
      V[c] = vv;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) p[j] = p[j] * decay - o.lr * g[j];
    }
    W[c] = p;
  }
}

// Worker-side pull of a row-sparse table striped over P parameter servers (global row r
// lives at local row r / P of PS r % P): every PS's stripe is an IPC-mapped peer pointer,
// so ONE launch gathers the rows of all owners over xGMI (no host-side owner split).
// tabs[p] / nrows[p]: device arrays of the P stripe pointers and their row counts.
template <bool OUT_BF16>
__global__ __launch_bounds__(kRowBlock) void embed_gather_striped_kernel(const uint64_t* __restrict__ tabs,
                                                                         const int64_t* __restrict__ nrows, int P,
                                                                         const int64_t* __restrict__ idx, int64_t n,
                                                                         int dim, void* __restrict__ out) {
  const int64_t r = (int64_t)blockIdx.x * (kRowBlock / kWave) + (threadIdx.x >> 6);
  if (r >= n) return;
  const int lane = threadIdx.x & 63;
  const int64_t id = idx[r];
  const int owner = id >= 0 ? (int)(id % P) : 0;
  const int64_t local = id >= 0 ? id / P : -1;
  const bool ok = id >= 0 && local < nrows[owner];
  const float* table = reinterpret_cast<const float*>(tabs[owner]);
  const f32x4* src = reinterpret_cast<const f32x4*>(table + (ok ? local : 0) * (int64_t)dim);
  const int d4 = dim >> 2;
  for (int c = lane; c < d4; c += kWave) {
    f32x4 v = ok ? src[c] : f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (OUT_BF16) {
      u32x2 o{pack2(v[0], v[1]), pack2(v[2], v[3])};
      reinterpret_cast<u32x2*>(static_cast<bf16_t*>(out) + r * (int64_t)dim)[c] = o;
    } else {
      reinterpret_cast<f32x4*>(static_cast<float*>(out) + r * (int64_t)dim)[c] = v;
    }
  }
}

// Worker-side sparse push: unique global ids [n] + fp32 row gradients [n, dim] are split by
// owner on the device and written straight into each PS's inbox (peer writes over xGMI):
// inbox_ids[p][pos] = id / P, inbox_grad[p][pos, :] = grad row.  pos comes from a per-owner
// counter in LOCAL memory (cnt, zeroed by the caller); sparse_push_counts_kernel then
// publishes the counts into the inboxes.  Row order inside an inbox is arbitrary (ids are
// unique, the update is per row).  Rows past `cap` are dropped (the host checks n <= cap).
__global__ __launch_bounds__(kRowBlock) void sparse_split_push_kernel(const int64_t* __restrict__ ids,
                                                                      const float* __restrict__ grad, int64_t n,
                                                                      int dim, int P,
                                                                      const uint64_t* __restrict__ inbox_ids,
                                                                      const uint64_t* __restrict__ inbox_grad,
                                                                      int* __restrict__ cnt, int64_t cap) {
  const int64_t r = (int64_t)blockIdx.x * (kRowBlock / kWave) + (threadIdx.x >> 6);
  if (r >= n) return;
  const int lane = threadIdx.x & 63;
  const int64_t id = ids[r];
  if (id < 0) return;
  const int owner = (int)(id % P);
  int pos = 0;
  if (lane == 0) pos = atomicAdd(cnt + owner, 1);
  pos = __shfl(pos, 0);
  if (pos >= cap) return;
  if (lane == 0) reinterpret_cast<int64_t*>(inbox_ids[owner])[pos] = id / P;
  const f32x4* src = reinterpret_cast<const f32x4*>(grad + r * (int64_t)dim);
  f32x4* dst = reinterpret_cast<f32x4*>(reinterpret_cast<float*>(inbox_grad[owner]) + (int64_t)pos * dim);
  for (int c = lane; c < (dim >> 2); c += kWave) dst[c] = src[c];
}

__global__ void sparse_push_counts_kernel(const int* __restrict__ cnt, int P, const uint64_t* __restrict__ inbox_cnt,
                                          int64_t cap) {
  const int p = threadIdx.x;
  if (p < P) *reinterpret_cast<int*>(inbox_cnt[p]) = (int)min((int64_t)cnt[p], cap);
}

// Push ordering on the device.  The worker's stream, after its inbox
// writes, runs ps_signal: a system-scope release store of the push sequence number into a
// flag word in the PS's HBM (IPC-mapped).  The PS's stream runs ps_wait before the update
// that reads the inboxes: one thread spins on a system-scope acquire load of that word,
// bounded by a wall-clock deadline (a worker killed between enqueue and execution must not
// wedge the PS's stream); a give-up is recorded in status[0] and the update is then skipped
// by the host (it reads the status after the update's event).
__global__ void ps_signal_kernel(uint32_t* __restrict__ flag, uint32_t value) {
  __threadfence_system();   // the inbox writes of the kernels before this one, past the L2
  __hip_atomic_store(flag, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void ps_wait_kernel(const uint32_t* __restrict__ flag, uint32_t value, uint64_t timeout_ticks,
                               int* __restrict__ status) {
  const uint64_t t0 = wall_clock64();
  while ((int32_t)(__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - value) < 0) {
    if (wall_clock64() - t0 > timeout_ticks) {
      __hip_atomic_store(status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

// fp32 src (possibly a peer's IPC-mapped shard) -> bf16 dst, 8 elements per lane-iteration.
__global__ __launch_bounds__(256) void pull_cast_kernel(const float* __restrict__ src, bf16_t* __restrict__ dst,
                                                        int64_t n8) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += stride) {
    const f32x4 a = reinterpret_cast<const f32x4*>(src)[2 * i];
    const f32x4 b = reinterpret_cast<const f32x4*>(src)[2 * i + 1];
    reinterpret_cast<u32x4*>(dst)[i] = u32x4{pack2(a[0], a[1]), pack2(a[2], a[3]), pack2(b[0], b[1]),
                                             pack2(b[2], b[3])};
  }
}

inline int row_blocks(int64_t n) { return (int)((n + (kRowBlock / kWave) - 1) / (kRowBlock / kWave)); }

// One tensor of a multi-tensor copy.  kind: 0 = local fp32, 1 = local bf16,
// 2 = no local tensor (push: write zeros).
struct PsEntry {
  uint64_t local;   // worker tensor (device pointer)
  int64_t off;      // element offset in the PS flat buffer (multiple of 4)
  int64_t numel;
  int32_t kind;
  int32_t pad;
};

constexpr int kMcThreads = 256;
constexpr int kMcChunk = kMcThreads * 4 * 8;   // elements per workgroup: 8 x 4-element steps per thread

// PUSH: flat[off + i] = fp32(local[i]);  PULL: local[i] = cast(flat[off + i]).
template <bool PUSH>
__global__ __launch_bounds__(kMcThreads) void ps_multi_copy_kernel(const PsEntry* __restrict__ tab,
                                                                   const int64_t* __restrict__ bstart, int n,
                                                                   float* __restrict__ flat) {
  // entry e owns workgroups [bstart[e], bstart[e+1])
  int lo = 0, hi = n;
  const int64_t b = blockIdx.x;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (bstart[mid] <= b) lo = mid; else hi = mid;
  }
  const PsEntry e = tab[lo];
  const int64_t c0 = (b - bstart[lo]) * kMcChunk;
  const int64_t c1 = min(e.numel, c0 + kMcChunk);
  float* f = flat + e.off;
  const int64_t v1 = c1 & ~int64_t(3);   // 4-element vectors (16 B fp32 / 8 B bf16)
  for (int64_t i = c0 + 4 * threadIdx.x; i < v1; i += 4 * kMcThreads) {
    if (PUSH) {
      f32x4 v;
      if (e.kind == 0) {
        v = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(e.local) + i);
      } else if (e.kind == 1) {
        const u32x2 w = *reinterpret_cast<const u32x2*>(reinterpret_cast<const bf16_t*>(e.local) + i);
        v = f32x4{__uint_as_float(w[0] << 16), __uint_as_float(w[0] & 0xffff0000u), __uint_as_float(w[1] << 16),
                  __uint_as_float(w[1] & 0xffff0000u)};
      } else {
        v = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      *reinterpret_cast<f32x4*>(f + i) = v;
    } else {
      const f32x4 v = *reinterpret_cast<const f32x4*>(f + i);
      if (e.kind == 0) {
        *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(e.local) + i) = v;
      } else if (e.kind == 1) {
        *reinterpret_cast<u32x2*>(reinterpret_cast<bf16_t*>(e.local) + i) = u32x2{pack2(v[0], v[1]), pack2(v[2], v[3])};
      }
    }
  }
  // tail of the tensor (numel % 4): scalar, in the last chunk only
  for (int64_t i = v1 + threadIdx.x; i < c1; i += kMcThreads) {
    if (PUSH) {
      float x = 0.f;
      if (e.kind == 0) x = reinterpret_cast<const float*>(e.local)[i];
      else if (e.kind == 1) x = bf2f(reinterpret_cast<const bf16_t*>(e.local)[i]);
      f[i] = x;
    } else {
      if (e.kind == 0) reinterpret_cast<float*>(e.local)[i] = f[i];
      else if (e.kind == 1) reinterpret_cast<bf16_t*>(e.local)[i] = f2bf(f[i]);
    }
  }
}

}  // namespace

extern "C" {

int edl_ps_multi_chunk() { return kMcChunk; }

// table / bstart: device arrays built by the host (easydl_amd/ops/sparse.py
// MultiCopyPlan); nblocks = bstart[n].  Local bf16 / fp32 tensors must be 8- /
// 16-byte aligned and every PS offset a multiple of 4 elements.
int edl_ps_multi_copy(const void* table, const int64_t* bstart, int n, int64_t nblocks, float* flat, int push,
                      hipStream_t s) {
  if (n <= 0 || nblocks <= 0) return 0;
  if (nblocks > 0x7fffffff) return (int)hipErrorInvalidValue;
  if (push)
    ps_multi_copy_kernel<true><<<(unsigned)nblocks, kMcThreads, 0, s>>>((const PsEntry*)table, bstart, n, flat);
  else
    ps_multi_copy_kernel<false><<<(unsigned)nblocks, kMcThreads, 0, s>>>((const PsEntry*)table, bstart, n, flat);
  EDL_LAUNCH_CHECK();
  return 0;
}

int edl_embed_gather(const float* table, const int64_t* idx, int64_t n, int dim, int64_t rows, void* out,
                     int out_bf16, hipStream_t s) {
  if (dim % 4 || n < 0 || rows < 1) return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  if (out_bf16)
    embed_gather_kernel<true><<<row_blocks(n), kRowBlock, 0, s>>>(table, idx, n, dim, rows, out);
  else
    embed_gather_kernel<false><<<row_blocks(n), kRowBlock, 0, s>>>(table, idx, n, dim, rows, out);
  EDL_LAUNCH_CHECK();
  return 0;
}

int edl_embed_scatter_add(float* acc, const int64_t* idx, const void* grad, int grad_bf16, int64_t n, int dim,
                          int64_t rows, hipStream_t s) {
  if (dim % 4 || n < 0 || rows < 1) return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  if (grad_bf16)
    embed_scatter_add_kernel<true><<<row_blocks(n), kRowBlock, 0, s>>>(acc, idx, grad, n, dim, rows);
  else
    embed_scatter_add_kernel<false><<<row_blocks(n), kRowBlock, 0, s>>>(acc, idx, grad, n, dim, rows);
  EDL_LAUNCH_CHECK();
  return 0;
}

// kind: 0 AdamW (m, v required), 1 Adagrad (v required), 2 SGD.  `step` is the
// table's update count after this update (bias correction of lazy Adam).
int edl_sparse_rows_update(float* w, float* m, float* v, const int64_t* rows_idx, const float* grad, int64_t nu,
                           int dim, int64_t rows, int kind, float lr, float beta1, float beta2, float eps, float wd,
                           int64_t step, float scale, hipStream_t s) {
  if (dim % 4 || nu < 0 || kind < 0 || kind > 2) return (int)hipErrorInvalidValue;
  if ((kind == 0 && (!m || !v)) || (kind == 1 && !v)) return (int)hipErrorInvalidValue;
  if (nu == 0) return 0;
  SparseOpt o{kind, lr, beta1, beta2, eps, wd, lr, 1.f, scale};
  if (kind == 0) {
    o.step_size = lr / (1.f - powf(beta1, (float)step));
    o.inv_bc2_sqrt = 1.f / sqrtf(1.f - powf(beta2, (float)step));
  }
  sparse_rows_update_kernel<<<row_blocks(nu), kRowBlock, 0, s>>>(w, m, v, rows_idx, grad, nu, dim, rows, o);
  EDL_LAUNCH_CHECK();
  return 0;
}

int edl_embed_gather_striped(const uint64_t* tabs, const int64_t* nrows, int P, const int64_t* idx, int64_t n,
                             int dim, void* out, int out_bf16, hipStream_t s) {
  if (dim % 4 || n < 0 || P < 1) return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  if (out_bf16)
    embed_gather_striped_kernel<true><<<row_blocks(n), kRowBlock, 0, s>>>(tabs, nrows, P, idx, n, dim, out);
  else
    embed_gather_striped_kernel<false><<<row_blocks(n), kRowBlock, 0, s>>>(tabs, nrows, P, idx, n, dim, out);
  EDL_LAUNCH_CHECK();
  return 0;
}

// cnt: P int32 of local scratch (zeroed here); inbox_* : device arrays of P peer pointers
int edl_sparse_split_push(const int64_t* ids, const float* grad, int64_t n, int dim, int P, const uint64_t* inbox_ids,
                          const uint64_t* inbox_grad, const uint64_t* inbox_cnt, int* cnt, int64_t cap,
                          hipStream_t s) {
  if (dim % 4 || n < 0 || P < 1 || P > 256 || n > cap) return (int)hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(cnt, 0, sizeof(int) * P, s);
  if (e != hipSuccess) return (int)e;
  if (n > 0)
    sparse_split_push_kernel<<<row_blocks(n), kRowBlock, 0, s>>>(ids, grad, n, dim, P, inbox_ids, inbox_grad, cnt,
                                                                  cap);
  EDL_LAUNCH_CHECK();
  sparse_push_counts_kernel<<<1, 256, 0, s>>>(cnt, P, inbox_cnt, cap);
  EDL_LAUNCH_CHECK();
  return 0;
}

int edl_sparse_inbox_update(float* w, float* m, float* v, const int64_t* ids, const float* grad, const int* count,
                            int64_t cap, int dim, int64_t rows, int kind, float lr, float beta1, float beta2, float eps,
                            float wd, int64_t step, float scale, hipStream_t s) {
  if (dim % 4 || cap < 0 || kind < 0 || kind > 2) return (int)hipErrorInvalidValue;
  if ((kind == 0 && (!m || !v)) || (kind == 1 && !v)) return (int)hipErrorInvalidValue;
  if (cap == 0) return 0;
  SparseOpt o{kind, lr, beta1, beta2, eps, wd, lr, 1.f, scale};
  if (kind == 0) {
    o.step_size = lr / (1.f - powf(beta1, (float)step));
    o.inv_bc2_sqrt = 1.f / sqrtf(1.f - powf(beta2, (float)step));
  }
  const int blocks = row_blocks(cap) < 1024 ? row_blocks(cap) : 1024;
  sparse_inbox_update_kernel<<<blocks, kRowBlock, 0, s>>>(w, m, v, ids, grad, count, cap, dim, rows, o);
  EDL_LAUNCH_CHECK();
  return 0;
}

int edl_ps_signal(uint32_t* flag, uint32_t value, hipStream_t s) {
  ps_signal_kernel<<<1, 1, 0, s>>>(flag, value);
  EDL_LAUNCH_CHECK();
  return 0;
}

int edl_ps_wait(const uint32_t* flag, uint32_t value, double timeout_s, int* status, hipStream_t s) {
  int dev = 0, khz = 0;
  hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0) khz = 100000;
  const uint64_t ticks = (uint64_t)(timeout_s * 1000.0 * (double)khz);
  ps_wait_kernel<<<1, 1, 0, s>>>(flag, value, ticks, status);
  EDL_LAUNCH_CHECK();
  return 0;
}

int edl_ps_pull_cast(const float* src, void* dst, int64_t n, hipStream_t s) {
  if (n % 8) return (int)hipErrorInvalidValue;
  const int64_t n8 = n / 8;
  if (n8 == 0) return 0;
  int64_t blocks = (n8 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  pull_cast_kernel<<<(int)blocks, 256, 0, s>>>(src, (bf16_t*)dst, n8);
  EDL_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
