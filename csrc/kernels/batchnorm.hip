// Training-mode BatchNorm over channels-last (NHWC) bf16 activations with the
// ReLU and the residual add of a ResNet bottleneck fused in:
//
//     z = relu?( (x - mean_c) * rstd_c * w_c + b_c  [+ r] )
//
// The activation is a row-major [M = N*H*W, C] matrix.  MIOpen's NHWC batch
// norm plus PyTorch's bf16<->fp32 casts, residual add and ReLU took 44 of the
// 63 ms of a ResNet-50 step at batch 256 on one MI355X (13 kernels per block);
// this is 2 passes forward (statistics; normalise+add+ReLU) and 2 backward
// (dbias/dweight reductions; dx [+ d residual]), each one streaming read of the
// bf16 tensors at 16 B per lane.
//
// Work split: a thread owns 8 consecutive channels (one 16-B vector) of a row;
// 256 / (C/8) rows of a block are read at once, so a block keeps its
// per-channel coefficients in registers for its whole row range.  The two
// reductions run on a (row block, channel chunk <= 256) grid, >= 256 rows per
// block, and a 1024-thread finalize sums the per-block partials per channel.
// Statistics are shifted by the running mean (sum (x - k), sum (x - k)^2 in
// fp32 per thread, fp64 across threads and blocks), so E[x^2] - E[x]^2 does not
// cancel once the running mean tracks the batch mean.  The backward sums
// dp * (x - mean) with the batch mean itself.
// Capability source: ResNet-50 bf16 elastic DDP (BASELINE.json config 2).
#include "common.h"

using namespace edl;

namespace {

constexpr int kThreads = 256;
constexpr int kFinThreads = 1024;
constexpr int kUnroll = 4;

// thread -> (8-channel group, row lane) inside a chunk of Cb channels; the chunk is
// blockIdx.y for the reductions (Cb = C for the elementwise kernels)
struct Geo {
  int tpr, rpi, col8, r0;
  bool active;
  __device__ __forceinline__ Geo(int Cb, int chunk) {
    tpr = Cb >> 3;
    rpi = kThreads / tpr;
    col8 = chunk * tpr + threadIdx.x % tpr;
    r0 = threadIdx.x / tpr;
    active = r0 < rpi;
  }
};

__device__ __forceinline__ void row_range(int64_t M, int rpi, int64_t& r, int64_t& end) {
  const int64_t per = ((M + gridDim.x - 1) / gridDim.x + rpi - 1) / rpi * rpi;
  r = (int64_t)blockIdx.x * per;
  end = min(M, r + per);
}

// Per-block column sums of two [rpi][Cb] fp32 register sets -> part[blockIdx.x][2][C]
// (this block's Cb channels)
__device__ __forceinline__ void block_colsum2(const float (&a)[8], const float (&b)[8], const Geo& g, int Cb,
                                              int C, float* part) {
  __shared__ float red[2][kThreads * 8];
  const int lc = (threadIdx.x % g.tpr) * 8;
  if (g.active) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[0][g.r0 * Cb + lc + j] = a[j];
      red[1][g.r0 * Cb + lc + j] = b[j];
    }
  }
  __syncthreads();
  float* out = part + (int64_t)blockIdx.x * 2 * C + blockIdx.y * Cb;
  for (int c = threadIdx.x; c < Cb; c += kThreads) {
    float s = 0.f, q = 0.f;
    for (int r = 0; r < g.rpi; ++r) {
      s += red[0][r * Cb + c];
      q += red[1][r * Cb + c];
    }
    out[c] = s;
    out[C + c] = q;
  }
}

// sum over the G row-block partials of channel c: 16 lanes of a 1024-thread block per
// channel, 4 independent fp64 chains per lane, then an LDS tree
__device__ __forceinline__ void sum_partials(const float* __restrict__ part, int G, int C, double& s, double& q) {
  __shared__ double red[2][kFinThreads];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), gl = threadIdx.x >> 6;
  double s4[4] = {}, q4[4] = {};
  if (c < C) {
    int i = gl;
    for (; i + 48 < G; i += 64) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        s4[u] += (double)part[(int64_t)(i + 16 * u) * 2 * C + c];
        q4[u] += (double)part[(int64_t)(i + 16 * u) * 2 * C + C + c];
      }
    }
    for (; i < G; i += 16) {
      s4[0] += (double)part[(int64_t)i * 2 * C + c];
      q4[0] += (double)part[(int64_t)i * 2 * C + C + c];
    }
  }
  red[0][threadIdx.x] = (s4[0] + s4[1]) + (s4[2] + s4[3]);
  red[1][threadIdx.x] = (q4[0] + q4[1]) + (q4[2] + q4[3]);
  __syncthreads();
  for (int w = kFinThreads / 2; w >= 64; w >>= 1) {
    if (threadIdx.x < w) {
      red[0][threadIdx.x] += red[0][threadIdx.x + w];
      red[1][threadIdx.x] += red[1][threadIdx.x + w];
    }
    __syncthreads();
  }
  s = red[0][threadIdx.x & 63];
  q = red[1][threadIdx.x & 63];
}

__device__ __forceinline__ void load8f(const float* p, float (&f)[8]) {
  const f32x4 a = *reinterpret_cast<const f32x4*>(p), b = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    f[j] = a[j];
    f[4 + j] = b[j];
  }
}

// ---------------------------------------------------------------------------- forward
__global__ __launch_bounds__(kThreads) void bn_stats_kernel(const bf16_t* __restrict__ x,
                                                            const float* __restrict__ shift, int64_t M, int C,
                                                            int Cb, float* __restrict__ part) {
  const Geo g(Cb, blockIdx.y);
  float s[8] = {}, q[8] = {};
  if (g.active) {
    float k[8];
    load8f(shift + g.col8 * 8, k);
    int64_t r, end;
    row_range(M, g.rpi, r, end);
    r += g.r0;
    const bf16_t* px = x + g.col8 * 8;
    for (; r + (kUnroll - 1) * g.rpi < end; r += kUnroll * g.rpi) {
      u32x4 v[kUnroll];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) v[u] = *reinterpret_cast<const u32x4*>(px + (r + u * g.rpi) * C);
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        float f[8];
        unpack8(v[u], f);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = f[j] - k[j];
          s[j] += d;
          q[j] = __builtin_fmaf(d, d, q[j]);
        }
      }
    }
    for (; r < end; r += g.rpi) {
      float f[8];
      unpack8(*reinterpret_cast<const u32x4*>(px + r * C), f);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = f[j] - k[j];
        s[j] += d;
        q[j] = __builtin_fmaf(d, d, q[j]);
      }
    }
  }
  block_colsum2(s, q, g, Cb, C, part);
}

// per channel: fp64 sum of the partials -> mean, rstd, affine coefficients, running stats
__global__ __launch_bounds__(kFinThreads) void bn_stats_finalize_kernel(
    const float* __restrict__ part, int G, int C, int64_t M, const float* __restrict__ w,
    const float* __restrict__ b, float* __restrict__ run_mean, float* __restrict__ run_var, float momentum,
    float eps, float* __restrict__ mean_out, float* __restrict__ rstd_out, float* __restrict__ coef,
    int64_t* __restrict__ nbt) {
  double s, q;
  sum_partials(part, G, C, s, q);
  const int c = blockIdx.x * 64 + threadIdx.x;
  if (nbt != nullptr && c == 0) nbt[0] += 1;   // the module's num_batches_tracked (no separate launch)
  if (threadIdx.x >= 64 || c >= C) return;
  const double k = (double)run_mean[c];
  const double dm = s / (double)M;
  const double var = fmax(q / (double)M - dm * dm, 0.0);
  const float mean = (float)(k + dm);
  const float rstd = (float)(1.0 / sqrt(var + (double)eps));
  mean_out[c] = mean;
  rstd_out[c] = rstd;
  const float sc = w[c] * rstd;
  coef[c] = sc;                 // z = x * sc + sh
  coef[C + c] = b[c] - mean * sc;
  run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * mean;
  const double unbiased = M > 1 ? var * (double)M / (double)(M - 1) : var;
  run_var[c] = (1.f - momentum) * run_var[c] + momentum * (float)unbiased;
}

template <bool RES, bool RELU>
__global__ __launch_bounds__(kThreads) void bn_apply_kernel(const bf16_t* __restrict__ x,
                                                            const bf16_t* __restrict__ res,
                                                            const float* __restrict__ coef, int64_t M, int C,
                                                            bf16_t* __restrict__ z) {
  const Geo g(C, 0);
  if (!g.active) return;
  float sc[8], sh[8];
  load8f(coef + g.col8 * 8, sc);
  load8f(coef + C + g.col8 * 8, sh);
  int64_t r, end;
  row_range(M, g.rpi, r, end);
  const int64_t o0 = g.col8 * 8;
  for (r += g.r0; r < end; r += g.rpi) {
    const int64_t o = r * C + o0;
    float f[8];
    unpack8(*reinterpret_cast<const u32x4*>(x + o), f);
    float e[8];
    if (RES) unpack8(*reinterpret_cast<const u32x4*>(res + o), e);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float v = __builtin_fmaf(f[j], sc[j], sh[j]);
      if (RES) v += e[j];
      if (RELU) v = fmaxf(v, 0.f);
      f[j] = v;
    }
    *reinterpret_cast<u32x4*>(z + o) = pack8(f);
  }
}

// ---------------------------------------------------------------------------- backward
// d += dz2, rounded to bf16 exactly as the separate bf16 add it replaces would store it
__device__ __forceinline__ void add_rounded(float (&d)[8], const u32x4& v2) {
  float e[8];
  unpack8(v2, e);
#pragma unroll
  for (int j = 0; j < 8; ++j) d[j] += e[j];
  unpack8(pack8(d), d);
}

// dp = relu ? (z > 0 ? dz : 0) : dz;   partials of sum dp and sum dp * (x - mean)
// MX: no residual was added, so the ReLU mask is recomputed from x with the forward's
// own coefficients (z > 0  <=>  fma(x, sc, sh) > 0) instead of reading z back from HBM
// D2: the output's gradient arrives in two parts, dz + dz2 (a ResNet block output's
// identity-path gradient, parked by the next block instead of summed by an add kernel)
template <bool RELU, bool MX, bool D2 = false>
__global__ __launch_bounds__(kThreads) void bn_bwd_reduce_kernel(const bf16_t* __restrict__ dz,
                                                                 const bf16_t* __restrict__ dz2,
                                                                 const bf16_t* __restrict__ z,
                                                                 const bf16_t* __restrict__ x,
                                                                 const float* __restrict__ mean,
                                                                 const float* __restrict__ fcoef, int64_t M, int C,
                                                                 int Cb, float* __restrict__ part) {
  const Geo g(Cb, blockIdx.y);
  float s[8] = {}, q[8] = {};
  if (g.active) {
    float mu[8], sc[8], sh[8];
    load8f(mean + g.col8 * 8, mu);
    if (MX) {
      load8f(fcoef + g.col8 * 8, sc);
      load8f(fcoef + C + g.col8 * 8, sh);
    }
    int64_t r, end;
    row_range(M, g.rpi, r, end);
    const int64_t o0 = g.col8 * 8;
    for (r += g.r0; r < end; r += g.rpi) {
      const int64_t o = r * C + o0;
      float d[8], f[8], y[8];
      unpack8(*reinterpret_cast<const u32x4*>(dz + o), d);
      unpack8(*reinterpret_cast<const u32x4*>(x + o), f);
      if (RELU && !MX) unpack8(*reinterpret_cast<const u32x4*>(z + o), y);
      if (D2) add_rounded(d, *reinterpret_cast<const u32x4*>(dz2 + o));
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (MX) y[j] = __builtin_fmaf(f[j], sc[j], sh[j]);
        const float dp = RELU ? (y[j] > 0.f ? d[j] : 0.f) : d[j];
        s[j] += dp;
        q[j] = __builtin_fmaf(dp, f[j] - mu[j], q[j]);
      }
    }
  }
  block_colsum2(s, q, g, Cb, C, part);
}

// dbias = sum dp, dweight = rstd * sum dp (x - mean); dx = A dp - K1 x + K2 with
// A = w rstd, K1 = w rstd^2 dweight / M, K2 = K1 mean - A dbias / M
__global__ __launch_bounds__(kFinThreads) void bn_bwd_finalize_kernel(const float* __restrict__ part, int G, int C,
                                                                      int64_t M, const float* __restrict__ w,
                                                                      const float* __restrict__ mean,
                                                                      const float* __restrict__ rstd,
                                                                      float* __restrict__ dw, float* __restrict__ db,
                                                                      float* __restrict__ coef, int acc) {
  double s, q;
  sum_partials(part, G, C, s, q);
  const int c = blockIdx.x * 64 + threadIdx.x;
  if (threadIdx.x >= 64 || c >= C) return;
  const double rs = (double)rstd[c];
  const double gw = q * rs, gb = s;
  // acc: dw / db are views of a flat gradient buffer that already holds earlier
  // micro-batches' gradients (no separate autograd accumulate launch per parameter)
  dw[c] = acc ? dw[c] + (float)gw : (float)gw;
  db[c] = acc ? db[c] + (float)gb : (float)gb;
  const double A = (double)w[c] * rs;
  const double K1 = A * rs * gw / (double)M;
  coef[c] = (float)A;
  coef[C + c] = (float)K1;
  coef[2 * C + c] = (float)(K1 * (double)mean[c] - A * gb / (double)M);
}

template <bool RELU, bool DRES, bool MX, bool D2 = false>
__global__ __launch_bounds__(kThreads) void bn_bwd_dx_kernel(const bf16_t* __restrict__ dz,
                                                             const bf16_t* __restrict__ dz2,
                                                             const bf16_t* __restrict__ z,
                                                             const bf16_t* __restrict__ x,
                                                             const float* __restrict__ coef,
                                                             const float* __restrict__ fcoef, int64_t M, int C,
                                                             bf16_t* __restrict__ dx, bf16_t* __restrict__ dres) {
  const Geo g(C, 0);
  if (!g.active) return;
  float A[8], K1[8], K2[8], sc[8], sh[8];
  load8f(coef + g.col8 * 8, A);
  load8f(coef + C + g.col8 * 8, K1);
  load8f(coef + 2 * C + g.col8 * 8, K2);
  if (MX) {
    load8f(fcoef + g.col8 * 8, sc);
    load8f(fcoef + C + g.col8 * 8, sh);
  }
  int64_t r, end;
  row_range(M, g.rpi, r, end);
  const int64_t o0 = g.col8 * 8;
  for (r += g.r0; r < end; r += g.rpi) {
    const int64_t o = r * C + o0;
    float d[8], f[8], y[8];
    unpack8(*reinterpret_cast<const u32x4*>(dz + o), d);
    unpack8(*reinterpret_cast<const u32x4*>(x + o), f);
    if (RELU && !MX) unpack8(*reinterpret_cast<const u32x4*>(z + o), y);
    if (D2) add_rounded(d, *reinterpret_cast<const u32x4*>(dz2 + o));
    float gx[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (MX) y[j] = __builtin_fmaf(f[j], sc[j], sh[j]);
      const float dp = RELU ? (y[j] > 0.f ? d[j] : 0.f) : d[j];
      d[j] = dp;
      gx[j] = __builtin_fmaf(A[j], dp, __builtin_fmaf(-K1[j], f[j], K2[j]));
    }
    *reinterpret_cast<u32x4*>(dx + o) = pack8(gx);
    if (DRES) *reinterpret_cast<u32x4*>(dres + o) = pack8(d);
  }
}

int blocks_for(int64_t M, int C, int min_rows_per_thread, int cap) {
  const int rpi = kThreads / (C >> 3);
  const int64_t want = (M + (int64_t)rpi * min_rows_per_thread - 1) / ((int64_t)rpi * min_rows_per_thread);
  return (int)(want < 1 ? 1 : want > cap ? cap : want);
}

bool shape_ok(int64_t M, int C) { return M > 0 && C >= 8 && C % 8 == 0 && C <= 8 * kThreads; }

// channel chunk of a reduction block: at most 32 8-channel groups (>= 8 rows per pass)
int chunk_of(int C) {
  const int t = C >> 3;
  int d = t <= 32 ? t : 32;
  while (t % d) --d;
  return 8 * d;
}

// row blocks of a reduction: >= 256 rows each (the [2][C] partial stays < 1 % of the
// data), <= ~1024 blocks over all channel chunks
int row_blocks(int64_t M, int C) {
  const int cc = C / chunk_of(C);
  const int64_t cap = 1024 / cc > 0 ? 1024 / cc : 1;
  const int64_t want = (M + 255) / 256;
  return (int)(want < 1 ? 1 : want > cap ? cap : want);
}

}  // namespace

extern "C" {

// partial-sum slab size of the reductions: floats = 2 * C * edl_bn_groups(M, C)
int edl_bn_groups(int64_t M, int C) { return shape_ok(M, C) ? row_blocks(M, C) : 0; }

// statistics + normalise (+ residual) (+ ReLU).  mean/rstd: fp32 [C] saved for the backward;
// coef: fp32 [2C] scratch; part: fp32 [2C * edl_bn_groups].  running_mean is also the shift.
int edl_bn_fwd_train(const void* x, const void* res, void* z, const float* w, const float* b, float* run_mean,
                     float* run_var, float* mean, float* rstd, float* coef, float* part, int64_t M, int C,
                     float momentum, float eps, int relu, int64_t* nbt, hipStream_t s) {
  if (!shape_ok(M, C)) return (int)hipErrorInvalidValue;
  const int G = row_blocks(M, C), Cb = chunk_of(C);
  bn_stats_kernel<<<dim3(G, C / Cb), kThreads, 0, s>>>((const bf16_t*)x, run_mean, M, C, Cb, part);
  EDL_LAUNCH_CHECK();
  bn_stats_finalize_kernel<<<(C + 63) / 64, kFinThreads, 0, s>>>(part, G, C, M, w, b, run_mean, run_var,
                                                                  momentum, eps, mean, rstd, coef, nbt);
  EDL_LAUNCH_CHECK();
  const int GA = blocks_for(M, C, 4, 2048);
#define EDL_BN_APPLY(R, L)                                                                               \
  bn_apply_kernel<R, L><<<GA, kThreads, 0, s>>>((const bf16_t*)x, (const bf16_t*)res, coef, M, C, (bf16_t*)z)
  if (res) {
    if (relu) EDL_BN_APPLY(true, true); else EDL_BN_APPLY(true, false);
  } else {
    if (relu) EDL_BN_APPLY(false, true); else EDL_BN_APPLY(false, false);
  }
#undef EDL_BN_APPLY
  EDL_LAUNCH_CHECK();
  return 0;
}

// z = x * coef[c] + coef[C + c] (+ res) (+ ReLU): eval mode, coef from the running statistics
int edl_bn_apply(const void* x, const void* res, void* z, const float* coef, int64_t M, int C, int relu,
                 hipStream_t s) {
  if (!shape_ok(M, C)) return (int)hipErrorInvalidValue;
  const int GA = blocks_for(M, C, 4, 2048);
  if (res) {
    if (relu)
      bn_apply_kernel<true, true><<<GA, kThreads, 0, s>>>((const bf16_t*)x, (const bf16_t*)res, coef, M, C,
                                                          (bf16_t*)z);
    else
      bn_apply_kernel<true, false><<<GA, kThreads, 0, s>>>((const bf16_t*)x, (const bf16_t*)res, coef, M, C,
                                                           (bf16_t*)z);
  } else {
    if (relu)
      bn_apply_kernel<false, true><<<GA, kThreads, 0, s>>>((const bf16_t*)x, nullptr, coef, M, C, (bf16_t*)z);
    else
      bn_apply_kernel<false, false><<<GA, kThreads, 0, s>>>((const bf16_t*)x, nullptr, coef, M, C, (bf16_t*)z);
  }
  EDL_LAUNCH_CHECK();
  return 0;
}

// dz (and z for the ReLU mask), x, saved mean/rstd -> dx, optional d residual, dw, db (fp32 [C]).
// coef: fp32 [3C] scratch; part as in the forward.
// fcoef: the forward's (scale, shift) coefficients [2C]; with relu and z == nullptr the
// ReLU mask is recomputed from x (forward without a residual), saving a read of z per pass
// dz2 (may be null): a second part of the output gradient, added in both passes (only with
// relu and z given: the block-output BatchNorm of a ResNet bottleneck)
int edl_bn_bwd(const void* dz, const void* dz2, const void* z, const void* x, const float* w, const float* mean,
               const float* rstd, const float* fcoef, void* dx, void* dres, float* dw, float* db, float* coef,
               float* part, int64_t M, int C, int relu, int acc, hipStream_t s) {
  if (!shape_ok(M, C) || (relu && z == nullptr && fcoef == nullptr)) return (int)hipErrorInvalidValue;
  if (dz2 && !(relu && z)) return (int)hipErrorInvalidValue;
  const bool mx = relu && z == nullptr;
  const int G = row_blocks(M, C), Cb = chunk_of(C);
  const dim3 grid(G, C / Cb);
  const bf16_t *bdz = (const bf16_t*)dz, *bdz2 = (const bf16_t*)dz2, *bz = (const bf16_t*)z, *bx = (const bf16_t*)x;
  if (mx)
    bn_bwd_reduce_kernel<true, true><<<grid, kThreads, 0, s>>>(bdz, nullptr, nullptr, bx, mean, fcoef, M, C, Cb, part);
  else if (relu && dz2)
    bn_bwd_reduce_kernel<true, false, true><<<grid, kThreads, 0, s>>>(bdz, bdz2, bz, bx, mean, nullptr, M, C, Cb, part);
  else if (relu)
    bn_bwd_reduce_kernel<true, false><<<grid, kThreads, 0, s>>>(bdz, nullptr, bz, bx, mean, nullptr, M, C, Cb, part);
  else
    bn_bwd_reduce_kernel<false, false><<<grid, kThreads, 0, s>>>(bdz, nullptr, nullptr, bx, mean, nullptr, M, C, Cb,
                                                                 part);
  EDL_LAUNCH_CHECK();
  bn_bwd_finalize_kernel<<<(C + 63) / 64, kFinThreads, 0, s>>>(part, G, C, M, w, mean, rstd, dw, db, coef, acc);
  EDL_LAUNCH_CHECK();
  const int GA = blocks_for(M, C, 4, 2048);
#define EDL_BN_DX(L, D, X, D2)                                                                    \
  bn_bwd_dx_kernel<L, D, X, D2><<<GA, kThreads, 0, s>>>(bdz, bdz2, bz, bx, coef, fcoef, M, C, (bf16_t*)dx, \
                                                        (bf16_t*)dres)
  if (dz2) {
    if (dres) EDL_BN_DX(true, true, false, true); else EDL_BN_DX(true, false, false, true);
  } else if (dres) {
    if (mx) EDL_BN_DX(true, true, true, false); else if (relu) EDL_BN_DX(true, true, false, false);
    else EDL_BN_DX(false, true, false, false);
  } else {
    if (mx) EDL_BN_DX(true, false, true, false); else if (relu) EDL_BN_DX(true, false, false, false);
    else EDL_BN_DX(false, false, false, false);
  }
#undef EDL_BN_DX
  EDL_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
