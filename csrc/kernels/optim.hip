// Fused optimizer kernels over FLAT parameter storage.
//
// easydl_amd keeps every parameter of a group as a view into ONE contiguous
// buffer (easydl_amd/parallel/flat.py), so the whole AdamW update of an
// 8B-parameter model is a single grid-stride launch — no multi-tensor
// metadata, no per-tensor launches.  Bytes per element (bf16 param, fp32
// master/m/v, bf16 grad): 2+4+4+4 read, 2+4+4+4 written = 28 B, i.e. the
// kernel is HBM-bound; each lane moves 4 elements per iteration with 8/16 B
// accesses (Guideline 13).
//
// The gradient scale (1/world for summed DDP grads x clip coefficient) is read
// from DEVICE memory written by edl_clip_finalize, so clipping needs no host
// synchronisation.  A non-finite flag set by the same kernel skips the update
// entirely (fault-tolerance hook: a poisoned step is dropped on every rank).
//
// Capability source: SURVEY.md §2.4 N4/N7 (fused AdamW, multi-tensor
// L2 norm + clip); the reference itself ships no kernels.
#include <type_traits>

#include "common.h"

using namespace edl;

namespace {

struct AdamArgs {
  float lr, beta1, beta2, eps, wd;
  float step_size;    // lr / (1 - beta1^t)
  float inv_bc2_sqrt; // 1 / sqrt(1 - beta2^t)
  float scale;        // host-side grad scale
};

template <typename G>
__device__ __forceinline__ void load4(const G* g, int64_t i, float (&o)[4]);
template <>
__device__ __forceinline__ void load4<bf16_t>(const bf16_t* g, int64_t i, float (&o)[4]) {
  u32x2 w = reinterpret_cast<const u32x2*>(g)[i];
  o[0] = bflo(w[0]); o[1] = bfhi(w[0]); o[2] = bflo(w[1]); o[3] = bfhi(w[1]);
}
template <>
__device__ __forceinline__ void load4<float>(const float* g, int64_t i, float (&o)[4]) {
  f32x4 w = reinterpret_cast<const f32x4*>(g)[i];
  o[0] = w[0]; o[1] = w[1]; o[2] = w[2]; o[3] = w[3];
}

// p16 may be null (fp32-only parameters: master IS the parameter).
template <typename G>
__global__ __launch_bounds__(256) void adamw_flat_kernel(bf16_t* __restrict__ p16, float* __restrict__ w,
                                                         float* __restrict__ m, float* __restrict__ v,
                                                         const G* __restrict__ g, int64_t n4, AdamArgs a,
                                                         const float* __restrict__ dscale) {
  float scale = a.scale;
  if (dscale) {
    if (dscale[2] != 0.f) return;  // non-finite gradients: skip the step
    scale *= dscale[0];
  }
  const float decay = 1.f - a.lr * a.wd;
  const float omb1 = 1.f - a.beta1, omb2 = 1.f - a.beta2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float gr[4];
    load4<G>(g, i, gr);
    f32x4 wv = reinterpret_cast<const f32x4*>(w)[i];
    f32x4 mv = reinterpret_cast<const f32x4*>(m)[i];
    f32x4 vv = reinterpret_cast<const f32x4*>(v)[i];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float gk = gr[k] * scale;
      mv[k] = a.beta1 * mv[k] + omb1 * gk;
      vv[k] = a.beta2 * vv[k] + omb2 * gk * gk;
      const float denom = sqrtf(vv[k]) * a.inv_bc2_sqrt + a.eps;
      wv[k] = wv[k] * decay - a.step_size * (mv[k] / denom);
    }
    reinterpret_cast<f32x4*>(w)[i] = wv;
    reinterpret_cast<f32x4*>(m)[i] = mv;
    reinterpret_cast<f32x4*>(v)[i] = vv;
    if (p16) {
      u32x2 o;
      o[0] = pack2(wv[0], wv[1]);
      o[1] = pack2(wv[2], wv[3]);
      reinterpret_cast<u32x2*>(p16)[i] = o;
    }
  }
}

// AdamW with bf16 moments (m, v stored in bf16, computed in fp32): 22 instead of 28 B per
// element, and 8 instead of 12 B per parameter of optimizer state in HBM and in every
// in-memory snapshot -- what lets a Llama-3-70B TP=8 shard keep FULL snapshots (weights AND
// moments) in the host DRAM a rank gets (ckpt/manager.py _decide_mode).  The moments are
// rounded to bf16 STOCHASTICALLY, with the random bits a hash of (element, step, m|v):
// unbiased (an EMA increment below half a bf16 ulp is not lost on average, as it would be
// with round-to-nearest), and deterministic, so a resume from a snapshot replays the next
// update bit for bit.  The weight update itself uses the unrounded fp32 moments.
__device__ __forceinline__ uint32_t mix32(uint32_t x) {   // "lowbias32" integer hash
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint32_t f2bf_sr_bits(float f, uint32_t r) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u) return f2bf_bits(f);   // inf / NaN: not rounded
  return (u + (r & 0xffffu)) >> 16;
}

template <typename G>
__global__ __launch_bounds__(256) void adamw_flat_m16_kernel(bf16_t* __restrict__ p16, float* __restrict__ w,
                                                             bf16_t* __restrict__ m, bf16_t* __restrict__ v,
                                                             const G* __restrict__ g, int64_t n4, AdamArgs a,
                                                             const float* __restrict__ dscale, uint32_t seed_m,
                                                             uint32_t seed_v) {
  float scale = a.scale;
  if (dscale) {
    if (dscale[2] != 0.f) return;
    scale *= dscale[0];
  }
  const float decay = 1.f - a.lr * a.wd;
  const float omb1 = 1.f - a.beta1, omb2 = 1.f - a.beta2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float gr[4];
    load4<G>(g, i, gr);
    f32x4 wv = reinterpret_cast<const f32x4*>(w)[i];
    const u32x2 mw = reinterpret_cast<const u32x2*>(m)[i];
    const u32x2 vw = reinterpret_cast<const u32x2*>(v)[i];
    float mk[4] = {bflo(mw[0]), bfhi(mw[0]), bflo(mw[1]), bfhi(mw[1])};
    float vk[4] = {bflo(vw[0]), bfhi(vw[0]), bflo(vw[1]), bfhi(vw[1])};
    uint32_t mo[4], vo[4];
    const uint32_t e0 = (uint32_t)(i * 4) * 0x9E3779B1u;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float gk = gr[k] * scale;
      mk[k] = a.beta1 * mk[k] + omb1 * gk;
      vk[k] = a.beta2 * vk[k] + omb2 * gk * gk;
      const float denom = sqrtf(vk[k]) * a.inv_bc2_sqrt + a.eps;
      wv[k] = wv[k] * decay - a.step_size * (mk[k] / denom);
      const uint32_t e = e0 + (uint32_t)k * 0x9E3779B1u;
      mo[k] = f2bf_sr_bits(mk[k], mix32(e + seed_m));
      vo[k] = f2bf_sr_bits(vk[k], mix32(e + seed_v));
    }
    reinterpret_cast<f32x4*>(w)[i] = wv;
    u32x2 om, ov;
    om[0] = mo[0] | (mo[1] << 16); om[1] = mo[2] | (mo[3] << 16);
    ov[0] = vo[0] | (vo[1] << 16); ov[1] = vo[2] | (vo[3] << 16);
    reinterpret_cast<u32x2*>(m)[i] = om;
    reinterpret_cast<u32x2*>(v)[i] = ov;
    if (p16) {
      u32x2 o;
      o[0] = pack2(wv[0], wv[1]);
      o[1] = pack2(wv[2], wv[3]);
      reinterpret_cast<u32x2*>(p16)[i] = o;
    }
  }
}

// Plain SGD with momentum over flat storage (used by the parameter server and
// ResNet recipes). mom may be null (no momentum).
template <typename G>
__global__ __launch_bounds__(256) void sgd_flat_kernel(bf16_t* __restrict__ p16, float* __restrict__ w,
                                                       float* __restrict__ mom, const G* __restrict__ g,
                                                       int64_t n4, float lr, float momentum, float wd,
                                                       float scale, const float* __restrict__ dscale) {
  if (dscale) {
    if (dscale[2] != 0.f) return;
    scale *= dscale[0];
  }
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float gr[4];
    load4<G>(g, i, gr);
    f32x4 wv = reinterpret_cast<const f32x4*>(w)[i];
    f32x4 mv = {0.f, 0.f, 0.f, 0.f};
    if (mom) mv = reinterpret_cast<const f32x4*>(mom)[i];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float d = gr[k] * scale + wd * wv[k];
      if (mom) { mv[k] = momentum * mv[k] + d; d = mv[k]; }
      wv[k] -= lr * d;
    }
    reinterpret_cast<f32x4*>(w)[i] = wv;
    if (mom) reinterpret_cast<f32x4*>(mom)[i] = mv;
    if (p16) {
      u32x2 o;
      o[0] = pack2(wv[0], wv[1]);
      o[1] = pack2(wv[2], wv[3]);
      reinterpret_cast<u32x2*>(p16)[i] = o;
    }
  }
}

// Per-block partial sum of squares; partial[blockIdx] (one float per block).
template <typename G>
__global__ __launch_bounds__(256) void sumsq_partial_kernel(const G* __restrict__ g, int64_t n4,
                                                            float* __restrict__ partial) {
  __shared__ float red[4];
  float acc = 0.f;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool wide = false;
  if constexpr (std::is_same_v<G, bf16_t>) wide = (reinterpret_cast<uintptr_t>(g) & 15) == 0;
  if (wide) {
    // bf16: 16-byte loads, four in flight per thread (the 8-byte, one-deep loop read 16 GB
    // of Llama-3-8B gradients at 3.7 TB/s)
    const int64_t n8 = n4 >> 1;
    const u32x4* g8 = reinterpret_cast<const u32x4*>(g);
    float a[4] = {0.f, 0.f, 0.f, 0.f};
    for (; i + 3 * stride < n8; i += 4 * stride) {
      u32x4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = g8[i + u * stride];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float f[8];
        unpack8(v[u], f);
#pragma unroll
        for (int k = 0; k < 8; ++k) a[u] += f[k] * f[k];
      }
    }
    for (; i < n8; i += stride) {
      float f[8];
      unpack8(g8[i], f);
#pragma unroll
      for (int k = 0; k < 8; ++k) a[0] += f[k] * f[k];
    }
    acc = (a[0] + a[1]) + (a[2] + a[3]);
    if ((n4 & 1) && blockIdx.x == 0 && threadIdx.x == 0) {   // odd 4-element tail
      float gr[4];
      load4<G>(g, n4 - 1, gr);
      acc += gr[0] * gr[0] + gr[1] * gr[1] + gr[2] * gr[2] + gr[3] * gr[3];
    }
  } else {
    for (; i < n4; i += stride) {
      float gr[4];
      load4<G>(g, i, gr);
      acc += gr[0] * gr[0] + gr[1] * gr[1] + gr[2] * gr[2] + gr[3] * gr[3];
    }
  }
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = acc;
}

// out[0] = combined grad scale (pre_scale * clip coefficient), out[1] = global
// grad norm (of the pre-scaled gradient), out[2] = 1 if non-finite else 0.
__global__ __launch_bounds__(256) void clip_finalize_kernel(const float* __restrict__ partial, int nparts,
                                                            float pre_scale, float max_norm,
                                                            float* __restrict__ out) {
  __shared__ double red[4];
  double acc = 0.0;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) acc += (double)partial[i];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += red[i];
    const float norm = (float)sqrt(t) * pre_scale;
    const bool bad = !isfinite(norm);
    float coef = pre_scale;
    if (max_norm > 0.f && norm > max_norm) coef = pre_scale * (max_norm / (norm + 1e-6f));
    out[0] = coef;
    out[1] = norm;
    out[2] = bad ? 1.f : 0.f;
  }
}

inline int grid_for(int64_t n4, int cap = 2048) {
  // EDL_ADAMW_GRID: fewer workgroups for the grid-stride update kernels, e.g. while they overlap
  // the next forward on another stream (read once per process)
  static const int env_cap = [] {
    const char* e = getenv("EDL_ADAMW_GRID");
    return e && atoi(e) > 0 ? atoi(e) : 0;
  }();
  if (env_cap > 0 && env_cap < cap) cap = env_cap;
  int64_t b = (n4 + 255) / 256;
  if (b < 1) b = 1;
  return (int)(b < cap ? b : cap);
}

}  // namespace

extern "C" {

// gdtype: 0 = bf16 grads, 1 = fp32 grads. n must be a multiple of 4 and all
// pointers 16-byte aligned (flat buffers are padded; checked in Python).
int edl_adamw_flat(void* p16, float* w, float* m, float* v, const void* g, int gdtype, int64_t n, float lr,
                   float beta1, float beta2, float eps, float wd, int64_t step, float scale,
                   const float* dscale, hipStream_t stream) {
  if (n % 4) return (int)hipErrorInvalidValue;
  AdamArgs a;
  a.lr = lr; a.beta1 = beta1; a.beta2 = beta2; a.eps = eps; a.wd = wd; a.scale = scale;
  const double bc1 = 1.0 - pow((double)beta1, (double)step);
  const double bc2 = 1.0 - pow((double)beta2, (double)step);
  a.step_size = (float)(lr / bc1);
  a.inv_bc2_sqrt = (float)(1.0 / sqrt(bc2));
  const int64_t n4 = n / 4;
  if (n4 == 0) return 0;
  const int grid = grid_for(n4);
  if (gdtype == 0)
    adamw_flat_kernel<bf16_t><<<grid, 256, 0, stream>>>((bf16_t*)p16, w, m, v, (const bf16_t*)g, n4, a, dscale);
  else
    adamw_flat_kernel<float><<<grid, 256, 0, stream>>>((bf16_t*)p16, w, m, v, (const float*)g, n4, a, dscale);
  EDL_LAUNCH_CHECK();
  return 0;
}

// bf16 moments (see adamw_flat_m16_kernel); seeds: (uint32)step * 0x85EBCA77 + salt (m / v).
int edl_adamw_flat_m16(void* p16, float* w, void* m, void* v, const void* g, int gdtype, int64_t n, float lr,
                       float beta1, float beta2, float eps, float wd, int64_t step, float scale,
                       const float* dscale, hipStream_t stream) {
  if (n % 4) return (int)hipErrorInvalidValue;
  AdamArgs a;
  a.lr = lr; a.beta1 = beta1; a.beta2 = beta2; a.eps = eps; a.wd = wd; a.scale = scale;
  const double bc1 = 1.0 - pow((double)beta1, (double)step);
  const double bc2 = 1.0 - pow((double)beta2, (double)step);
  a.step_size = (float)(lr / bc1);
  a.inv_bc2_sqrt = (float)(1.0 / sqrt(bc2));
  const int64_t n4 = n / 4;
  if (n4 == 0) return 0;
  const uint32_t base = (uint32_t)step * 0x85EBCA77u;
  const uint32_t seed_m = base + 0x27d4eb2fu, seed_v = base + 0x165667b1u;
  const int grid = grid_for(n4);
  if (gdtype == 0)
    adamw_flat_m16_kernel<bf16_t><<<grid, 256, 0, stream>>>((bf16_t*)p16, w, (bf16_t*)m, (bf16_t*)v,
                                                            (const bf16_t*)g, n4, a, dscale, seed_m, seed_v);
  else
    adamw_flat_m16_kernel<float><<<grid, 256, 0, stream>>>((bf16_t*)p16, w, (bf16_t*)m, (bf16_t*)v,
                                                           (const float*)g, n4, a, dscale, seed_m, seed_v);
  EDL_LAUNCH_CHECK();
  return 0;
}

int edl_sgd_flat(void* p16, float* w, float* mom, const void* g, int gdtype, int64_t n, float lr, float momentum,
                 float wd, float scale, const float* dscale, hipStream_t stream) {
  if (n % 4) return (int)hipErrorInvalidValue;
  const int64_t n4 = n / 4;
  if (n4 == 0) return 0;
  const int grid = grid_for(n4);
  if (gdtype == 0)
    sgd_flat_kernel<bf16_t><<<grid, 256, 0, stream>>>((bf16_t*)p16, w, mom, (const bf16_t*)g, n4, lr, momentum, wd,
                                                      scale, dscale);
  else
    sgd_flat_kernel<float><<<grid, 256, 0, stream>>>((bf16_t*)p16, w, mom, (const float*)g, n4, lr, momentum, wd,
                                                     scale, dscale);
  EDL_LAUNCH_CHECK();
  return 0;
}

// Number of partials edl_sumsq_partial writes for n elements.
int edl_sumsq_nparts(int64_t n) { return grid_for(n / 4, 1024); }

int edl_sumsq_partial(const void* g, int gdtype, int64_t n, float* partial, hipStream_t stream) {
  if (n % 4) return (int)hipErrorInvalidValue;
  const int64_t n4 = n / 4;
  const int grid = grid_for(n4, 1024);
  if (gdtype == 0)
    sumsq_partial_kernel<bf16_t><<<grid, 256, 0, stream>>>((const bf16_t*)g, n4, partial);
  else
    sumsq_partial_kernel<float><<<grid, 256, 0, stream>>>((const float*)g, n4, partial);
  EDL_LAUNCH_CHECK();
  return 0;
}

int edl_clip_finalize(const float* partial, int nparts, float pre_scale, float max_norm, float* out,
                      hipStream_t stream) {
  clip_finalize_kernel<<<1, 256, 0, stream>>>(partial, nparts, pre_scale, max_norm, out);
  EDL_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
