// Fused elementwise kernels of the transformer block:
//   * SwiGLU over the packed [gate | up] output of ONE fused gate+up GEMM
//   * RoPE + QKV split: the fused QKV GEMM output [T, (H+2KV)*D] is rotated and
//     split into q [T,H*D], k [T,KV*D], v [T,KV*D] in one pass (the [B,S,H,D]
//     memory layout that flash attention consumes without a copy); the
//     backward applies the inverse rotation and re-packs d(qkv).
//   * Softmax cross-entropy fwd+bwd in one kernel over the [T, V] logits:
//     loss per row, and the logits buffer is overwritten IN PLACE with
//     softmax - onehot (vocab 128256 bf16 logits are 2 GB at 8k tokens; no
//     second buffer is allocated).
// All kernels move 16 B per lane (8 bf16) per access.
//
// Capability source: Llama-3 workloads of BASELINE.json configs 3 and 5
// (SURVEY.md §2.9); the reference ships no kernels.
#include "common.h"

using namespace edl;

namespace {

// ---------------------------------------------------------------------------
// SwiGLU
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void swiglu_fwd_kernel(const bf16_t* __restrict__ gu, bf16_t* __restrict__ out,
                                                         int64_t rows, int F) {
  const int fc = F >> 3;
  const int64_t total = rows * fc;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += stride) {
    const int64_t r = e / fc;
    const int c = (int)(e - r * fc);
    const u32x4* row = reinterpret_cast<const u32x4*>(gu + r * 2 * F);
    float g[8], u[8], o[8];
    unpack8(row[c], g);
    unpack8(row[fc + c], u);
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = g[k] * sigmoidf_(g[k]) * u[k];
    reinterpret_cast<u32x4*>(out + r * F)[c] = pack8(o);
  }
}

__global__ __launch_bounds__(256) void swiglu_bwd_kernel(const bf16_t* __restrict__ dout,
                                                         const bf16_t* __restrict__ gu, bf16_t* __restrict__ dgu,
                                                         int64_t rows, int F) {
  const int fc = F >> 3;
  const int64_t total = rows * fc;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += stride) {
    const int64_t r = e / fc;
    const int c = (int)(e - r * fc);
    const u32x4* row = reinterpret_cast<const u32x4*>(gu + r * 2 * F);
    float g[8], u[8], d[8], dg[8], du[8];
    unpack8(row[c], g);
    unpack8(row[fc + c], u);
    unpack8(reinterpret_cast<const u32x4*>(dout + r * F)[c], d);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float s = sigmoidf_(g[k]);
      const float silu = g[k] * s;
      du[k] = d[k] * silu;
      dg[k] = d[k] * u[k] * s * (1.f + g[k] * (1.f - s));
    }
    u32x4* orow = reinterpret_cast<u32x4*>(dgu + r * 2 * F);
    orow[c] = pack8(dg);
    orow[fc + c] = pack8(du);
  }
}

// ---------------------------------------------------------------------------
// RoPE (rotate-half convention) fused with the QKV split.
// One work item = (token t, head h in [0, H+KV), chunk j in [0, D/16)):
// rotates elements [8j, 8j+8) with their partners [D/2+8j, D/2+8j+8).
// V heads are copied by work items (t, h in [H+KV, H+2KV), chunk j in [0, D/8)).
// ---------------------------------------------------------------------------
template <bool BWD>
__global__ __launch_bounds__(256) void rope_qkv_kernel(const bf16_t* __restrict__ src_qkv,  // fwd: [T,(H+2KV)D]
                                                       bf16_t* __restrict__ q, bf16_t* __restrict__ k,
                                                       bf16_t* __restrict__ v, bf16_t* __restrict__ dst_qkv,
                                                       const float* __restrict__ cos_t,
                                                       const float* __restrict__ sin_t,  // [S, D/2]
                                                       int64_t T, int S, int H, int KV, int D) {
  const int half = D >> 1;
  const int jr = half >> 3;  // rotate chunks per head
  const int jv = D >> 3;     // copy chunks per v head
  const int per_tok = (H + KV) * jr + KV * jv;
  const int64_t total = T * per_tok;
  const int W = (H + 2 * KV) * D;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += stride) {
    const int64_t t = e / per_tok;
    int r = (int)(e - t * per_tok);
    const int s = (int)(t % S);
    if (r < (H + KV) * jr) {
      const int h = r / jr, j = r - h * jr;
      bf16_t* dst;
      int64_t dst_off;
      if (h < H) { dst = q; dst_off = t * (int64_t)H * D + (int64_t)h * D; }
      else { dst = k; dst_off = t * (int64_t)KV * D + (int64_t)(h - H) * D; }
      const int64_t qkv_off = t * W + (int64_t)h * D;
      const f32x4* cp = reinterpret_cast<const f32x4*>(cos_t + (int64_t)s * half + j * 8);
      const f32x4* sp = reinterpret_cast<const f32x4*>(sin_t + (int64_t)s * half + j * 8);
      const f32x4 c0 = cp[0], c1 = cp[1], s0 = sp[0], s1 = sp[1];
      const float cs[8] = {c0[0], c0[1], c0[2], c0[3], c1[0], c1[1], c1[2], c1[3]};
      const float sn[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
      float a[8], b[8], oa[8], ob[8];
      if (!BWD) {
        unpack8(*reinterpret_cast<const u32x4*>(src_qkv + qkv_off + j * 8), a);
        unpack8(*reinterpret_cast<const u32x4*>(src_qkv + qkv_off + half + j * 8), b);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          oa[i] = a[i] * cs[i] - b[i] * sn[i];
          ob[i] = b[i] * cs[i] + a[i] * sn[i];
        }
        *reinterpret_cast<u32x4*>(dst + dst_off + j * 8) = pack8(oa);
        *reinterpret_cast<u32x4*>(dst + dst_off + half + j * 8) = pack8(ob);
      } else {
        unpack8(*reinterpret_cast<const u32x4*>(dst + dst_off + j * 8), a);
        unpack8(*reinterpret_cast<const u32x4*>(dst + dst_off + half + j * 8), b);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          oa[i] = a[i] * cs[i] + b[i] * sn[i];
          ob[i] = b[i] * cs[i] - a[i] * sn[i];
        }
        *reinterpret_cast<u32x4*>(dst_qkv + qkv_off + j * 8) = pack8(oa);
        *reinterpret_cast<u32x4*>(dst_qkv + qkv_off + half + j * 8) = pack8(ob);
      }
    } else {
      r -= (H + KV) * jr;
      const int h = r / jv, j = r - h * jv;
      const int64_t qkv_off = t * W + (int64_t)(H + KV + h) * D + j * 8;
      const int64_t v_off = t * (int64_t)KV * D + (int64_t)h * D + j * 8;
      if (!BWD)
        *reinterpret_cast<u32x4*>(v + v_off) = *reinterpret_cast<const u32x4*>(src_qkv + qkv_off);
      else
        *reinterpret_cast<u32x4*>(dst_qkv + qkv_off) = *reinterpret_cast<const u32x4*>(v + v_off);
    }
  }
}

// ---------------------------------------------------------------------------
// Cross-entropy: one 256-lane workgroup per row. Pass 1: online (max, sum-exp)
// over the row with 16-B loads + target logit. Pass 2 (re-read hits the
// Infinity Cache): grad = softmax - onehot written in place (unscaled; the
// autograd wrapper applies dloss / n_valid).  ignore_index rows get loss 0 and
// zero gradient.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void xent_fwd_bwd_kernel(bf16_t* __restrict__ logits,
                                                           const int64_t* __restrict__ labels,
                                                           float* __restrict__ loss, int V, int64_t ignore_index,
                                                           int write_grad, const float* __restrict__ gscale,
                                                           float* __restrict__ lse_out) {
  __shared__ float sm[4], ss[4];
  __shared__ float s_tgt;
  const int64_t row = blockIdx.x;
  bf16_t* lr = logits + row * (int64_t)V;
  const int64_t lab = labels[row];
  const bool ignored = (lab == ignore_index) || lab < 0 || lab >= V;
  const int nchunk = V >> 3;
  float m = -INFINITY, s = 0.f;
  const u32x4* lv = reinterpret_cast<const u32x4*>(lr);
  for (int c = threadIdx.x; c < nchunk; c += blockDim.x) {
    float f[8];
    unpack8(lv[c], f);
    float cm = f[0];
#pragma unroll
    for (int i = 1; i < 8; ++i) cm = fmaxf(cm, f[i]);
    const float nm = fmaxf(m, cm);
    float acc = s * __expf(m - nm);
#pragma unroll
    for (int i = 0; i < 8; ++i) acc += __expf(f[i] - nm);
    m = nm;
    s = acc;
  }
  for (int c = (nchunk << 3) + threadIdx.x; c < V; c += blockDim.x) {  // tail (V % 8)
    const float f = bf2f(lr[c]);
    const float nm = fmaxf(m, f);
    s = s * __expf(m - nm) + __expf(f - nm);
    m = nm;
  }
  // combine (m, s) across the wave, then across waves
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float om = __shfl_xor(m, off, 64), os = __shfl_xor(s, off, 64);
    const float nm = fmaxf(m, om);
    s = (m == -INFINITY ? 0.f : s * __expf(m - nm)) + (om == -INFINITY ? 0.f : os * __expf(om - nm));
    m = nm;
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if (lane == 0) { sm[wid] = m; ss[wid] = s; }
  if (threadIdx.x == 0) s_tgt = ignored ? 0.f : bf2f(lr[lab]);
  __syncthreads();
  float M = sm[0];
  for (int i = 1; i < nw; ++i) M = fmaxf(M, sm[i]);
  float Ssum = 0.f;
  for (int i = 0; i < nw; ++i) Ssum += ss[i] * __expf(sm[i] - M);
  const float lse = M + __logf(Ssum);
  if (threadIdx.x == 0) {
    loss[row] = ignored ? 0.f : (lse - s_tgt);
    if (lse_out) lse_out[row] = lse;
  }
  if (!write_grad) return;
  // gradient multiplier (device scalar, e.g. dloss / n_valid): the backward writes the
  // final gradient in one pass instead of a separate scaling pass over V x rows
  const float g = gscale ? *gscale : 1.f;
  const float inv = g / Ssum;
  u32x4* lw = reinterpret_cast<u32x4*>(lr);
  for (int c = threadIdx.x; c < nchunk; c += blockDim.x) {
    float f[8];
    unpack8(lw[c], f);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float p = ignored ? 0.f : __expf(f[i] - M) * inv;
      if (!ignored && (int64_t)(c * 8 + i) == lab) p -= g;
      f[i] = p;
    }
    lw[c] = pack8(f);
  }
  for (int c = (nchunk << 3) + threadIdx.x; c < V; c += blockDim.x) {
    float p = ignored ? 0.f : __expf(bf2f(lr[c]) - M) * inv;
    if (!ignored && (int64_t)c == lab) p -= g;
    lr[c] = f2bf(p);
  }
}

// Backward from the forward's per-row log-sum-exp: grad = (exp(x - lse) - onehot) * (*gscale)
// written in place -- one read + one write of the logits (the recomputing form above reads
// them twice).  ignore_index rows -> 0.
__global__ __launch_bounds__(256) void xent_grad_lse_kernel(bf16_t* __restrict__ logits,
                                                            const int64_t* __restrict__ labels,
                                                            const float* __restrict__ lse_in, int V,
                                                            int64_t ignore_index, const float* __restrict__ gscale) {
  const int64_t row = blockIdx.x;
  bf16_t* lr = logits + row * (int64_t)V;
  const int64_t lab = labels[row];
  const bool ignored = (lab == ignore_index) || lab < 0 || lab >= V;
  const float g = gscale ? *gscale : 1.f;
  const float lse = lse_in[row];
  const int nchunk = V >> 3;
  u32x4* lw = reinterpret_cast<u32x4*>(lr);
  for (int c = threadIdx.x; c < nchunk; c += blockDim.x) {
    float f[8];
    unpack8(lw[c], f);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float p = ignored ? 0.f : __expf(f[i] - lse) * g;
      if (!ignored && (int64_t)(c * 8 + i) == lab) p -= g;
      f[i] = p;
    }
    lw[c] = pack8(f);
  }
  for (int c = (nchunk << 3) + threadIdx.x; c < V; c += blockDim.x) {
    float p = ignored ? 0.f : __expf(bf2f(lr[c]) - lse) * g;
    if (!ignored && (int64_t)c == lab) p -= g;
    lr[c] = f2bf(p);
  }
}

// Vocab-parallel cross-entropy (tensor parallelism, easydl_amd/parallel/tp.py): this
// rank holds columns [vstart, vstart + V) of every row.
//   stats mode: st[row] = (local max m, local sum exp(x - m), logit of the label if
//     it falls in this shard else 0) -> the caller combines ranks with one MAX and
//     one SUM all-reduce of [rows] / [rows, 2] fp32 (never the logits);
//   grad mode: with the global (M, S) in gs[row] = (M, S), overwrite the logits in
//     place with (exp(x - M) / S - onehot) * (*gscale); ignored rows -> 0.
template <bool GRAD>
__global__ __launch_bounds__(256) void xent_vp_kernel(bf16_t* __restrict__ logits, const int64_t* __restrict__ labels,
                                                      float* __restrict__ st, int V, int64_t vstart,
                                                      int64_t ignore_index, const float* __restrict__ gscale) {
  const int64_t row = blockIdx.x;
  bf16_t* lr = logits + row * (int64_t)V;
  const int64_t lab = labels[row];
  const int64_t loc = lab - vstart;
  const bool ignored = lab == ignore_index;
  const bool here = !ignored && loc >= 0 && loc < V;
  const int nchunk = V >> 3;
  if (GRAD) {
    const float M = st[2 * row], S = st[2 * row + 1];
    const float g = gscale ? *gscale : 1.f;
    const float inv = g / S;
    u32x4* lw = reinterpret_cast<u32x4*>(lr);
    for (int c = threadIdx.x; c < nchunk; c += blockDim.x) {
      float f[8];
      unpack8(lw[c], f);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float p = ignored ? 0.f : __expf(f[i] - M) * inv;
        if (here && (int64_t)(c * 8 + i) == loc) p -= g;
        f[i] = p;
      }
      lw[c] = pack8(f);
    }
    for (int c = (nchunk << 3) + threadIdx.x; c < V; c += blockDim.x) {
      float p = ignored ? 0.f : __expf(bf2f(lr[c]) - M) * inv;
      if (here && (int64_t)c == loc) p -= g;
      lr[c] = f2bf(p);
    }
    return;
  }
  __shared__ float sm[4], ss[4];
  float m = -INFINITY, s = 0.f;
  const u32x4* lv = reinterpret_cast<const u32x4*>(lr);
  for (int c = threadIdx.x; c < nchunk; c += blockDim.x) {
    float f[8];
    unpack8(lv[c], f);
    float cm = f[0];
#pragma unroll
    for (int i = 1; i < 8; ++i) cm = fmaxf(cm, f[i]);
    const float nm = fmaxf(m, cm);
    float acc = s * __expf(m - nm);
#pragma unroll
    for (int i = 0; i < 8; ++i) acc += __expf(f[i] - nm);
    m = nm;
    s = acc;
  }
  for (int c = (nchunk << 3) + threadIdx.x; c < V; c += blockDim.x) {
    const float f = bf2f(lr[c]);
    const float nm = fmaxf(m, f);
    s = s * __expf(m - nm) + __expf(f - nm);
    m = nm;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float om = __shfl_xor(m, off, 64), os = __shfl_xor(s, off, 64);
    const float nm = fmaxf(m, om);
    s = (m == -INFINITY ? 0.f : s * __expf(m - nm)) + (om == -INFINITY ? 0.f : os * __expf(om - nm));
    m = nm;
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if (lane == 0) { sm[wid] = m; ss[wid] = s; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = sm[0];
    for (int i = 1; i < nw; ++i) M = fmaxf(M, sm[i]);
    float S = 0.f;
    for (int i = 0; i < nw; ++i) S += ss[i] * __expf(sm[i] - M);
    st[3 * row] = M;
    st[3 * row + 1] = S;
    st[3 * row + 2] = here ? bf2f(lr[loc]) : 0.f;
  }
}

// y = x * s[0] in place over bf16 (s is a device scalar: no host sync).
__global__ __launch_bounds__(256) void scale_bf16_kernel(bf16_t* __restrict__ x, int64_t n8,
                                                         const float* __restrict__ s, float hs) {
  const float sc = (s ? s[0] : 1.f) * hs;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += stride) {
    float f[8];
    u32x4* p = reinterpret_cast<u32x4*>(x);
    unpack8(p[i], f);
#pragma unroll
    for (int k = 0; k < 8; ++k) f[k] *= sc;
    p[i] = pack8(f);
  }
}

inline int grid_for(int64_t items, int cap = 4096) {
  int64_t b = (items + 255) / 256;
  if (b < 1) b = 1;
  return (int)(b < cap ? b : cap);
}


// bf16 [R, C] -> [C, R] through a padded 64x64 LDS tile: 16-B global loads along
// C, 16-B global stores along R (both coalesced); the LDS row stride of 66
// elements (33 banks) keeps the column reads of the transposed pass conflict-
// free.  HBM-bound: 4 B moved per element.  Used to keep a [in, out] copy of
// Linear weights so the input-gradient GEMM runs in hipBLASLt's fast NT form.
__global__ __launch_bounds__(256) void transpose_bf16_kernel(const bf16_t* __restrict__ src, bf16_t* __restrict__ dst,
                                                             int R, int C) {
  constexpr int T = 64, P = T + 2;
  __shared__ bf16_t tile[T * P];
  const int r0 = blockIdx.y * T, c0 = blockIdx.x * T;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int idx = threadIdx.x + 256 * i;      // 512 chunks of 8 elements
    const int r = idx >> 3, c8 = (idx & 7) * 8;
    const int gr = r0 + r, gc = c0 + c8;
    if (gr < R && gc + 8 <= C) {
      const u32x4 v = *reinterpret_cast<const u32x4*>(src + (int64_t)gr * C + gc);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        tile[r * P + c8 + 2 * j] = (bf16_t)(v[j] & 0xffffu);
        tile[r * P + c8 + 2 * j + 1] = (bf16_t)(v[j] >> 16);
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int idx = threadIdx.x + 256 * i;
    const int c = idx >> 3, r8 = (idx & 7) * 8;  // output row c, columns r8..r8+7
    const int gc = c0 + c, gr = r0 + r8;
    if (gc < C && gr + 8 <= R) {
      u32x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        o[j] = (uint32_t)tile[(r8 + 2 * j) * P + c] | ((uint32_t)tile[(r8 + 2 * j + 1) * P + c] << 16);
      *reinterpret_cast<u32x4*>(dst + (int64_t)gc * R + gr) = o;
    }
  }
}

// ---------------------------------------------------------------------------
// SwiGLU with a transposed copy of its output, for the NT-form weight gradients
// of the MLP (ops/fused.py::swiglu_mlp).  One workgroup = a 64-row x 64-column
// tile of h (fwd) or of d_gate/d_up (bwd).  The row-major result is written as
// usual; the same tile also goes through a padded LDS tile and out transposed
// (16-B stores along the token axis).  Writing the transposed copy here costs
// one extra write; a separate transpose kernel would read it back and write it.
// ---------------------------------------------------------------------------
constexpr int TT = 64, TP = TT + 2;

// column c of the tile, rows r8..r8+7, as one 16-B chunk
__device__ __forceinline__ u32x4 tile_col8(const bf16_t* tile, int c, int r8) {
  u32x4 o;
#pragma unroll
  for (int j = 0; j < 4; ++j)
    o[j] = (uint32_t)tile[(r8 + 2 * j) * TP + c] | ((uint32_t)tile[(r8 + 2 * j + 1) * TP + c] << 16);
  return o;
}

// gu [M, 2F] -> h [M, F] and hT [F, M]
__global__ __launch_bounds__(256) void swiglu_fwd_t_kernel(const bf16_t* __restrict__ gu, bf16_t* __restrict__ h,
                                                           bf16_t* __restrict__ hT, int M, int F) {
  __shared__ bf16_t tile[TT * TP];
  const int r0 = blockIdx.y * TT, c0 = blockIdx.x * TT;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int idx = threadIdx.x + 256 * i;
    const int r = idx >> 3, c8 = (idx & 7) * 8;
    const int gr = r0 + r, gc = c0 + c8;
    if (gr < M && gc + 8 <= F) {
      const bf16_t* row = gu + (int64_t)gr * 2 * F;
      float g[8], u[8], o[8];
      unpack8(*reinterpret_cast<const u32x4*>(row + gc), g);
      unpack8(*reinterpret_cast<const u32x4*>(row + F + gc), u);
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = g[k] * sigmoidf_(g[k]) * u[k];
      const u32x4 packed = pack8(o);
      *reinterpret_cast<u32x4*>(h + (int64_t)gr * F + gc) = packed;
#pragma unroll
      for (int j = 0; j < 4; ++j) {   // the bf16 values exactly as stored in h
        tile[r * TP + c8 + 2 * j] = (bf16_t)(packed[j] & 0xffffu);
        tile[r * TP + c8 + 2 * j + 1] = (bf16_t)(packed[j] >> 16);
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int idx = threadIdx.x + 256 * i;
    const int c = idx >> 3, r8 = (idx & 7) * 8;
    const int gc = c0 + c, gr = r0 + r8;
    if (gc < F && gr + 8 <= M) *reinterpret_cast<u32x4*>(hT + (int64_t)gc * M + gr) = tile_col8(tile, c, r8);
  }
}

// dh [M, F], gu [M, 2F] -> dgu [M, 2F] and dguT [2F, M]
__global__ __launch_bounds__(256) void swiglu_bwd_t_kernel(const bf16_t* __restrict__ dh,
                                                           const bf16_t* __restrict__ gu, bf16_t* __restrict__ dgu,
                                                           bf16_t* __restrict__ dguT, int M, int F) {
  __shared__ bf16_t tg[TT * TP], tu[TT * TP];
  const int r0 = blockIdx.y * TT, c0 = blockIdx.x * TT;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int idx = threadIdx.x + 256 * i;
    const int r = idx >> 3, c8 = (idx & 7) * 8;
    const int gr = r0 + r, gc = c0 + c8;
    if (gr < M && gc + 8 <= F) {
      const bf16_t* row = gu + (int64_t)gr * 2 * F;
      float g[8], u[8], d[8], dg[8], du[8];
      unpack8(*reinterpret_cast<const u32x4*>(row + gc), g);
      unpack8(*reinterpret_cast<const u32x4*>(row + F + gc), u);
      unpack8(*reinterpret_cast<const u32x4*>(dh + (int64_t)gr * F + gc), d);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float sg = sigmoidf_(g[k]);
        du[k] = d[k] * g[k] * sg;
        dg[k] = d[k] * u[k] * sg * (1.f + g[k] * (1.f - sg));
      }
      const u32x4 pg = pack8(dg), pu = pack8(du);
      bf16_t* orow = dgu + (int64_t)gr * 2 * F;
      *reinterpret_cast<u32x4*>(orow + gc) = pg;
      *reinterpret_cast<u32x4*>(orow + F + gc) = pu;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        tg[r * TP + c8 + 2 * j] = (bf16_t)(pg[j] & 0xffffu);
        tg[r * TP + c8 + 2 * j + 1] = (bf16_t)(pg[j] >> 16);
        tu[r * TP + c8 + 2 * j] = (bf16_t)(pu[j] & 0xffffu);
        tu[r * TP + c8 + 2 * j + 1] = (bf16_t)(pu[j] >> 16);
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int idx = threadIdx.x + 256 * i;
    const int c = idx >> 3, r8 = (idx & 7) * 8;
    const int gc = c0 + c, gr = r0 + r8;
    if (gc < F && gr + 8 <= M) {
      *reinterpret_cast<u32x4*>(dguT + (int64_t)gc * M + gr) = tile_col8(tg, c, r8);
      *reinterpret_cast<u32x4*>(dguT + (int64_t)(F + gc) * M + gr) = tile_col8(tu, c, r8);
    }
  }
}

// ---------------------------------------------------------------------------
// Register-transposed forms (no LDS, no barrier).  Each lane owns an 8x8 bf16
// block: 8 row loads of 16 B, an in-register transpose (v_perm), 8 stores of
// 16 B along the other axis.  Lane = cb + 8 * rb inside a wave's 64x64 tile, so
// every load and every store instruction of a wave covers 8 full 128-B lines;
// a 256-thread block is a 128x128 tile (2x2 waves: 256 contiguous bytes per
// row on both sides).  8-24 independent 16-B loads in flight per lane instead
// of 2-6, and no 2-byte LDS traffic: the LDS versions above were
// instruction-bound at ~4.1-4.7 TB/s.
// ---------------------------------------------------------------------------
constexpr int RT = 128;  // block tile (rows and columns)

// out[j] = column j of the 8x8 block whose rows are in[0..7]
__device__ __forceinline__ void transpose8x8(const u32x4 (&in)[8], u32x4 (&out)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t a = in[2 * k][j >> 1], b = in[2 * k + 1][j >> 1];
      out[j][k] = (j & 1) ? ((a >> 16) | (b & 0xffff0000u)) : ((a & 0xffffu) | (b << 16));
    }
}

// this lane's 8x8 block origin (row, column) inside the grid's 128x128 tiles.
// Tiles are visited in diagonal order: consecutive (co-resident) workgroups
// step BOTH the row and the column tile, so neither their loads nor their
// transposed stores all sit at one power-of-two pitch (M = 16384 tokens is a
// 32 KB row pitch on the transposed side: row-major order camps on a few
// HBM channels).
__device__ __forceinline__ void block8_origin(int& r, int& c) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int gx = gridDim.x, gy = gridDim.y;
  const int b = blockIdx.x + gx * blockIdx.y;
  const int ty = b % gy, tx = (b / gy + ty) % gx;
  r = ty * RT + (w >> 1) * 64 + (lane >> 3) * 8;
  c = tx * RT + (w & 1) * 64 + (lane & 7) * 8;
}

__global__ __launch_bounds__(256) void transpose_bf16_reg_kernel(const bf16_t* __restrict__ src,
                                                                 bf16_t* __restrict__ dst, int R, int C) {
  int r, c;
  block8_origin(r, c);
  if (r >= R || c >= C) return;  // R, C multiples of 8: a block is all in or all out
  u32x4 in[8], out[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) in[i] = *reinterpret_cast<const u32x4*>(src + (int64_t)(r + i) * C + c);
  transpose8x8(in, out);
#pragma unroll
  for (int j = 0; j < 8; ++j) *reinterpret_cast<u32x4*>(dst + (int64_t)(c + j) * R + r) = out[j];
}

// Many transposes in one launch (the per-step refresh of every cached W^T): one 128x128 tile
// per workgroup over the concatenated tile lists.  A BERT-large weight alone is 64-256
// tiles, too few for 256 CUs (9.4 us per 1024 x 1024 transpose as separate launches).
// Descriptor i = 4 int64: src, dst, (R << 32) | C, (first tile << 32) | column tiles.
__global__ __launch_bounds__(256) void transpose_bf16_multi_kernel(const int64_t* __restrict__ desc, int n) {
  const int b = blockIdx.x;
  int lo = 0, hi = n - 1;   // last descriptor whose first tile <= b (wave-uniform search)
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if ((int)(desc[4 * mid + 3] >> 32) <= b) lo = mid; else hi = mid - 1;
  }
  const int64_t* d = desc + 4 * lo;
  const bf16_t* src = reinterpret_cast<const bf16_t*>(d[0]);
  bf16_t* dst = reinterpret_cast<bf16_t*>(d[1]);
  const int R = (int)(d[2] >> 32), C = (int)(d[2] & 0xffffffff);
  const int local = b - (int)(d[3] >> 32), tx_n = (int)(d[3] & 0xffffffff);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = (local / tx_n) * RT + (w >> 1) * 64 + (lane >> 3) * 8;
  const int c = (local % tx_n) * RT + (w & 1) * 64 + (lane & 7) * 8;
  if (r >= R || c >= C) return;  // R, C multiples of 8: a block is all in or all out
  u32x4 in[8], out[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) in[i] = *reinterpret_cast<const u32x4*>(src + (int64_t)(r + i) * C + c);
  transpose8x8(in, out);
#pragma unroll
  for (int j = 0; j < 8; ++j) *reinterpret_cast<u32x4*>(dst + (int64_t)(c + j) * R + r) = out[j];
}

// Transpose + column sums of src (the bias gradient of a linear layer is the column
// sum of dY, whose transpose the NT weight-gradient GEMM needs anyway): each thread
// sums its 8x8 block's columns, the 16 row groups of a 128x128 tile meet in LDS, and
// the tile writes one row of a [R/128, C] fp32 slab that edl_colsum reduces
// (deterministic, no float atomics).
__global__ __launch_bounds__(256) void transpose_colsum_bf16_kernel(const bf16_t* __restrict__ src,
                                                                    bf16_t* __restrict__ dst,
                                                                    float* __restrict__ partial, int R, int C) {
  __shared__ float red[16][RT + 4];
  int r, c;
  block8_origin(r, c);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int rg = (w >> 1) * 8 + (lane >> 3), c0 = ((w & 1) * 8 + (lane & 7)) * 8;
  const bool live = r < R && c < C;   // R, C multiples of 8: a block is all in or all out
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (live) {
    u32x4 in[8], out[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      in[i] = *reinterpret_cast<const u32x4*>(src + (int64_t)(r + i) * C + c);
      float f[8];
      unpack8(in[i], f);
#pragma unroll
      for (int k = 0; k < 8; ++k) cs[k] += f[k];
    }
    transpose8x8(in, out);
#pragma unroll
    for (int j = 0; j < 8; ++j) *reinterpret_cast<u32x4*>(dst + (int64_t)(c + j) * R + r) = out[j];
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) red[rg][c0 + k] = cs[k];
  __syncthreads();
  if (threadIdx.x < RT) {
    // this tile's column origin and row-tile index (block8_origin's mapping, lane-independent part)
    const int gx = gridDim.x, gy = gridDim.y;
    const int b = blockIdx.x + gx * blockIdx.y;
    const int ty = b % gy, tx = (b / gy + ty) % gx;
    const int col = tx * RT + threadIdx.x;
    if (col < C) {
      float t = 0.f;
#pragma unroll
      for (int g = 0; g < 16; ++g) t += red[g][threadIdx.x];
      partial[(int64_t)ty * C + col] = t;
    }
  }
}

__global__ __launch_bounds__(256) void swiglu_fwd_t_reg_kernel(const bf16_t* __restrict__ gu, bf16_t* __restrict__ h,
                                                               bf16_t* __restrict__ hT, int M, int F) {
  int r, c;
  block8_origin(r, c);
  if (r >= M || c >= F) return;
  u32x4 g8[8], u8[8], o8[8], t8[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const bf16_t* row = gu + (int64_t)(r + i) * 2 * F;
    g8[i] = *reinterpret_cast<const u32x4*>(row + c);
    u8[i] = *reinterpret_cast<const u32x4*>(row + F + c);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    float g[8], u[8], o[8];
    unpack8(g8[i], g);
    unpack8(u8[i], u);
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = g[k] * sigmoidf_(g[k]) * u[k];
    o8[i] = pack8(o);
    *reinterpret_cast<u32x4*>(h + (int64_t)(r + i) * F + c) = o8[i];
  }
  transpose8x8(o8, t8);
#pragma unroll
  for (int j = 0; j < 8; ++j) *reinterpret_cast<u32x4*>(hT + (int64_t)(c + j) * M + r) = t8[j];
}

__global__ __launch_bounds__(256) void swiglu_bwd_t_reg_kernel(const bf16_t* __restrict__ dh,
                                                               const bf16_t* __restrict__ gu, bf16_t* __restrict__ dgu,
                                                               bf16_t* __restrict__ dguT, int M, int F) {
  int r, c;
  block8_origin(r, c);
  if (r >= M || c >= F) return;
  u32x4 a8[8], b8[8], d8[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const bf16_t* row = gu + (int64_t)(r + i) * 2 * F;
    a8[i] = *reinterpret_cast<const u32x4*>(row + c);
    b8[i] = *reinterpret_cast<const u32x4*>(row + F + c);
    d8[i] = *reinterpret_cast<const u32x4*>(dh + (int64_t)(r + i) * F + c);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {   // a8 <- d_gate, b8 <- d_up (same math as swiglu_bwd_t_kernel)
    float g[8], u[8], d[8], dg[8], du[8];
    unpack8(a8[i], g);
    unpack8(b8[i], u);
    unpack8(d8[i], d);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float sg = sigmoidf_(g[k]);
      du[k] = d[k] * g[k] * sg;
      dg[k] = d[k] * u[k] * sg * (1.f + g[k] * (1.f - sg));
    }
    a8[i] = pack8(dg);
    b8[i] = pack8(du);
    bf16_t* orow = dgu + (int64_t)(r + i) * 2 * F;
    *reinterpret_cast<u32x4*>(orow + c) = a8[i];
    *reinterpret_cast<u32x4*>(orow + F + c) = b8[i];
  }
  transpose8x8(a8, d8);
#pragma unroll
  for (int j = 0; j < 8; ++j) *reinterpret_cast<u32x4*>(dguT + (int64_t)(c + j) * M + r) = d8[j];
  transpose8x8(b8, d8);
#pragma unroll
  for (int j = 0; j < 8; ++j) *reinterpret_cast<u32x4*>(dguT + (int64_t)(F + c + j) * M + r) = d8[j];
}

// packed [T, 3, HD] q|k|v rows -> contiguous q, k, v [T, HD] in one pass (BERT: one
// launch instead of three strided copies); 8 bf16 per chunk, a chunk of each of q, k, v per iteration
__global__ __launch_bounds__(256) void qkv_split_kernel(const bf16_t* __restrict__ qkv, bf16_t* __restrict__ q,
                                                        bf16_t* __restrict__ k, bf16_t* __restrict__ v, int64_t T,
                                                        int hd8) {
  const int64_t n = T * hd8;   // chunks per output tensor
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t t = i / hd8;
    const int c = (int)(i - t * hd8);
    const u32x4* src = reinterpret_cast<const u32x4*>(qkv) + t * 3 * hd8 + c;
    reinterpret_cast<u32x4*>(q)[i] = src[0];
    if (k) reinterpret_cast<u32x4*>(k)[i] = src[hd8];   // k / v null: q only
    if (v) reinterpret_cast<u32x4*>(v)[i] = src[2 * hd8];
  }
}

// ---------------------------------------------------------------------------
// tanh-approximated GELU (BERT MLP) with the transposed operand the NT weight-
// gradient GEMM needs, same register-transposed 8x8 blocks as the SwiGLU pair.
// forward: h = gelu(u), hT = h^T.  backward: du = gelu'(u) * dh, duT = du^T and
// per-128-row-tile column sums of du (the fc1 bias gradient, reduced by
// edl_colsum) -- one pass replaces PyTorch's GELU kernels plus a separate
// transpose of h and a transpose + column sum of du.
// ---------------------------------------------------------------------------
constexpr float kGeluC = 0.7978845608028654f;   // sqrt(2 / pi)
constexpr float kGeluA = 0.044715f;

// tanh(z) = 1 - 2 / (e^2z + 1), saturating cleanly at +-inf; v_rcp_f32 (1 ulp) instead of an
// IEEE division (a ~10-instruction scale/fma/fixup sequence): these kernels are VALU-bound
// once the transposed copy is not written (BERT-large: 64 M elements per call)
__device__ __forceinline__ float tanh_fast_(float z) {
  return 1.f - 2.f * __builtin_amdgcn_rcpf(__expf(2.f * z) + 1.f);
}

__device__ __forceinline__ float gelu_tanh_(float u) {
  const float z = kGeluC * (u + kGeluA * u * u * u);
  const float t = tanh_fast_(z);
  return 0.5f * u * (1.f + t);
}

__device__ __forceinline__ float gelu_tanh_grad_(float u) {
  const float z = kGeluC * (u + kGeluA * u * u * u);
  const float t = tanh_fast_(z);
  return 0.5f * (1.f + t) + 0.5f * u * (1.f - t * t) * kGeluC * (1.f + 3.f * kGeluA * u * u);
}

__global__ __launch_bounds__(256) void gelu_fwd_t_reg_kernel(const bf16_t* __restrict__ u, bf16_t* __restrict__ h,
                                                             bf16_t* __restrict__ hT, int M, int F) {
  int r, c;
  block8_origin(r, c);
  if (r >= M || c >= F) return;
  u32x4 o8[8], t8[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) o8[i] = *reinterpret_cast<const u32x4*>(u + (int64_t)(r + i) * F + c);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    float x[8];
    unpack8(o8[i], x);
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = gelu_tanh_(x[k]);
    o8[i] = pack8(x);
    *reinterpret_cast<u32x4*>(h + (int64_t)(r + i) * F + c) = o8[i];
  }
  if (!hT) return;   // no transposed copy (weight gradient by the TN GEMM, gemm_tn.hip)
  transpose8x8(o8, t8);
#pragma unroll
  for (int j = 0; j < 8; ++j) *reinterpret_cast<u32x4*>(hT + (int64_t)(c + j) * M + r) = t8[j];
}

__global__ __launch_bounds__(256) void gelu_bwd_t_reg_kernel(const bf16_t* __restrict__ dh,
                                                             const bf16_t* __restrict__ u, bf16_t* __restrict__ du,
                                                             bf16_t* __restrict__ duT, float* __restrict__ partial,
                                                             int M, int F) {
  __shared__ float red[16][RT + 4];
  int r, c;
  block8_origin(r, c);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int rg = (w >> 1) * 8 + (lane >> 3), c0 = ((w & 1) * 8 + (lane & 7)) * 8;
  const bool live = r < M && c < F;   // M, F multiples of 8: a block is all in or all out
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (live) {
    u32x4 a8[8], d8[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      a8[i] = *reinterpret_cast<const u32x4*>(u + (int64_t)(r + i) * F + c);
      d8[i] = *reinterpret_cast<const u32x4*>(dh + (int64_t)(r + i) * F + c);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float x[8], d[8];
      unpack8(a8[i], x);
      unpack8(d8[i], d);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        x[k] = d[k] * gelu_tanh_grad_(x[k]);
        cs[k] += x[k];
      }
      a8[i] = pack8(x);
      *reinterpret_cast<u32x4*>(du + (int64_t)(r + i) * F + c) = a8[i];
    }
    if (duT) {   // null: no transposed copy (weight gradient by the TN GEMM)
      transpose8x8(a8, d8);
#pragma unroll
      for (int j = 0; j < 8; ++j) *reinterpret_cast<u32x4*>(duT + (int64_t)(c + j) * M + r) = d8[j];
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) red[rg][c0 + k] = cs[k];
  __syncthreads();
  if (threadIdx.x < RT) {   // this tile's column origin / row-tile index (block8_origin's mapping)
    const int gx = gridDim.x, gy = gridDim.y;
    const int b = blockIdx.x + gx * blockIdx.y;
    const int ty = b % gy, tx = (b / gy + ty) % gx;
    const int col = tx * RT + threadIdx.x;
    if (col < F) {
      float t = 0.f;
#pragma unroll
      for (int g = 0; g < 16; ++g) t += red[g][threadIdx.x];
      partial[(int64_t)ty * F + col] = t;
    }
  }
}

}  // namespace

extern "C" {

int edl_swiglu_fwd(const void* gu, void* out, int64_t rows, int F, hipStream_t s) {
  if (F % 8) return (int)hipErrorInvalidValue;
  swiglu_fwd_kernel<<<grid_for(rows * (F / 8)), 256, 0, s>>>((const bf16_t*)gu, (bf16_t*)out, rows, F);
  EDL_LAUNCH_CHECK();
  return 0;
}

int edl_swiglu_bwd(const void* dout, const void* gu, void* dgu, int64_t rows, int F, hipStream_t s) {
  if (F % 8) return (int)hipErrorInvalidValue;
  swiglu_bwd_kernel<<<grid_for(rows * (F / 8)), 256, 0, s>>>((const bf16_t*)dout, (const bf16_t*)gu,
                                                             (bf16_t*)dgu, rows, F);
  EDL_LAUNCH_CHECK();
  return 0;
}

// h = swiglu(gu) and hT = h^T (M, F multiples of 8)
int edl_swiglu_fwd_t(const void* gu, void* h, void* hT, int M, int F, hipStream_t s) {
  if (F % 8 || M % 8 || M <= 0 || F <= 0) return (int)hipErrorInvalidValue;
  dim3 grid((F + RT - 1) / RT, (M + RT - 1) / RT);
  swiglu_fwd_t_reg_kernel<<<grid, 256, 0, s>>>((const bf16_t*)gu, (bf16_t*)h, (bf16_t*)hT, M, F);
  EDL_LAUNCH_CHECK();
  return 0;
}

// LDS-tile version (kept for A/B measurement: scripts/transpose_ab.py)
int edl_swiglu_fwd_t_lds(const void* gu, void* h, void* hT, int M, int F, hipStream_t s) {
  if (F % 8 || M % 8 || M <= 0 || F <= 0) return (int)hipErrorInvalidValue;
  dim3 grid((F + TT - 1) / TT, (M + TT - 1) / TT);
  swiglu_fwd_t_kernel<<<grid, 256, 0, s>>>((const bf16_t*)gu, (bf16_t*)h, (bf16_t*)hT, M, F);
  EDL_LAUNCH_CHECK();
  return 0;
}

// dgu = swiglu'(gu) * dh and dguT = dgu^T
int edl_swiglu_bwd_t(const void* dh, const void* gu, void* dgu, void* dguT, int M, int F, hipStream_t s) {
  if (F % 8 || M % 8 || M <= 0 || F <= 0) return (int)hipErrorInvalidValue;
  dim3 grid((F + RT - 1) / RT, (M + RT - 1) / RT);
  swiglu_bwd_t_reg_kernel<<<grid, 256, 0, s>>>((const bf16_t*)dh, (const bf16_t*)gu, (bf16_t*)dgu,
                                               (bf16_t*)dguT, M, F);
  EDL_LAUNCH_CHECK();
  return 0;
}

int edl_swiglu_bwd_t_lds(const void* dh, const void* gu, void* dgu, void* dguT, int M, int F, hipStream_t s) {
  if (F % 8 || M % 8 || M <= 0 || F <= 0) return (int)hipErrorInvalidValue;
  dim3 grid((F + TT - 1) / TT, (M + TT - 1) / TT);
  swiglu_bwd_t_kernel<<<grid, 256, 0, s>>>((const bf16_t*)dh, (const bf16_t*)gu, (bf16_t*)dgu, (bf16_t*)dguT, M,
                                           F);
  EDL_LAUNCH_CHECK();
  return 0;
}

// q / k / v [T, HD] = slices of packed qkv [T, 3 * HD] (HD multiple of 8); k and v may be null (q only)
int edl_qkv_split(const void* qkv, void* q, void* k, void* v, int64_t T, int HD, hipStream_t s) {
  if (HD % 8 || T <= 0) return (int)hipErrorInvalidValue;
  qkv_split_kernel<<<grid_for(T * (HD / 8)), 256, 0, s>>>((const bf16_t*)qkv, (bf16_t*)q, (bf16_t*)k, (bf16_t*)v, T,
                                                          HD / 8);
  EDL_LAUNCH_CHECK();
  return 0;
}

// h = gelu_tanh(u) and hT = h^T (M, F multiples of 8; hT may be null: h only)
int edl_gelu_fwd_t(const void* u, void* h, void* hT, int M, int F, hipStream_t s) {
  if (F % 8 || M % 8 || M <= 0 || F <= 0) return (int)hipErrorInvalidValue;
  dim3 grid((F + RT - 1) / RT, (M + RT - 1) / RT);
  gelu_fwd_t_reg_kernel<<<grid, 256, 0, s>>>((const bf16_t*)u, (bf16_t*)h, (bf16_t*)hT, M, F);
  EDL_LAUNCH_CHECK();
  return 0;
}

// du = gelu_tanh'(u) * dh, duT = du^T (may be null), partial[edl_transpose_tiles(M), F] = column sums of du
int edl_gelu_bwd_t(const void* dh, const void* u, void* du, void* duT, float* partial, int M, int F,
                   hipStream_t s) {
  if (F % 8 || M % 8 || M <= 0 || F <= 0) return (int)hipErrorInvalidValue;
  dim3 grid((F + RT - 1) / RT, (M + RT - 1) / RT);
  gelu_bwd_t_reg_kernel<<<grid, 256, 0, s>>>((const bf16_t*)dh, (const bf16_t*)u, (bf16_t*)du, (bf16_t*)duT,
                                             partial, M, F);
  EDL_LAUNCH_CHECK();
  return 0;
}

int edl_rope_qkv_fwd(const void* qkv, void* q, void* k, void* v, const float* cos_t, const float* sin_t, int64_t T,
                     int S, int H, int KV, int D, hipStream_t s) {
  if (D % 16) return (int)hipErrorInvalidValue;
  const int64_t items = T * ((H + KV) * (D / 16) + KV * (D / 8));
  rope_qkv_kernel<false><<<grid_for(items), 256, 0, s>>>((const bf16_t*)qkv, (bf16_t*)q, (bf16_t*)k, (bf16_t*)v,
                                                         nullptr, cos_t, sin_t, T, S, H, KV, D);
  EDL_LAUNCH_CHECK();
  return 0;
}

int edl_rope_qkv_bwd(const void* dq, const void* dk, const void* dv, void* dqkv, const float* cos_t,
                     const float* sin_t, int64_t T, int S, int H, int KV, int D, hipStream_t s) {
  if (D % 16) return (int)hipErrorInvalidValue;
  const int64_t items = T * ((H + KV) * (D / 16) + KV * (D / 8));
  rope_qkv_kernel<true><<<grid_for(items), 256, 0, s>>>(nullptr, (bf16_t*)dq, (bf16_t*)dk, (bf16_t*)dv,
                                                        (bf16_t*)dqkv, cos_t, sin_t, T, S, H, KV, D);
  EDL_LAUNCH_CHECK();
  return 0;
}

// write_grad: overwrite logits with (softmax - onehot) * (*gscale) (gscale may be null = 1)
// lse_out (may be null): the per-row log-sum-exp, for edl_xent_grad_lse
int edl_xent_fwd_bwd(void* logits, const int64_t* labels, float* loss, int64_t rows, int V, int64_t ignore_index,
                     int write_grad, const float* gscale, float* lse_out, hipStream_t s) {
  if (rows <= 0) return 0;
  xent_fwd_bwd_kernel<<<(unsigned)rows, 256, 0, s>>>((bf16_t*)logits, labels, loss, V, ignore_index, write_grad,
                                                     gscale, lse_out);
  EDL_LAUNCH_CHECK();
  return 0;
}

// logits <- (softmax - onehot) * (*gscale) from the forward's lse (one read + one write)
int edl_xent_grad_lse(void* logits, const int64_t* labels, const float* lse, int64_t rows, int V,
                      int64_t ignore_index, const float* gscale, hipStream_t s) {
  if (rows <= 0) return 0;
  xent_grad_lse_kernel<<<(unsigned)rows, 256, 0, s>>>((bf16_t*)logits, labels, lse, V, ignore_index, gscale);
  EDL_LAUNCH_CHECK();
  return 0;
}

// vocab-parallel cross-entropy: grad = 0 -> st[rows, 3] = (local max, local sum, local target
// logit); grad = 1 -> logits <- (softmax(global M, S from st[rows, 2]) - onehot) * (*gscale)
int edl_xent_vp(void* logits, const int64_t* labels, float* st, int64_t rows, int V, int64_t vstart,
                int64_t ignore_index, int grad, const float* gscale, hipStream_t s) {
  if (rows <= 0) return 0;
  if (V % 8) return (int)hipErrorInvalidValue;
  if (grad)
    xent_vp_kernel<true><<<(unsigned)rows, 256, 0, s>>>((bf16_t*)logits, labels, st, V, vstart, ignore_index, gscale);
  else
    xent_vp_kernel<false><<<(unsigned)rows, 256, 0, s>>>((bf16_t*)logits, labels, st, V, vstart, ignore_index,
                                                         gscale);
  EDL_LAUNCH_CHECK();
  return 0;
}

// dst[C, R] = src[R, C]^T (bf16, R and C multiples of 8)
// n transposes in one launch; desc: device int64 [n, 4] (see transpose_bf16_multi_kernel),
// first tiles ascending, tiles = the total 128x128 tile count
int edl_transpose_bf16_multi(const void* desc, int n, int tiles, hipStream_t s) {
  if (n <= 0 || tiles <= 0) return (int)hipErrorInvalidValue;
  transpose_bf16_multi_kernel<<<tiles, 256, 0, s>>>((const int64_t*)desc, n);
  EDL_LAUNCH_CHECK();
  return 0;
}

int edl_transpose_bf16(const void* src, void* dst, int R, int C, hipStream_t s) {
  if (R % 8 || C % 8 || R <= 0 || C <= 0) return (int)hipErrorInvalidValue;
  dim3 grid((C + RT - 1) / RT, (R + RT - 1) / RT);
  transpose_bf16_reg_kernel<<<grid, 256, 0, s>>>((const bf16_t*)src, (bf16_t*)dst, R, C);
  EDL_LAUNCH_CHECK();
  return 0;
}

// dst = src^T and partial[R/128 (rounded up), C] = per-row-tile column sums of src (fp32)
int edl_transpose_colsum_bf16(const void* src, void* dst, float* partial, int R, int C, hipStream_t s) {
  if (R % 8 || C % 8 || R <= 0 || C <= 0) return (int)hipErrorInvalidValue;
  dim3 grid((C + RT - 1) / RT, (R + RT - 1) / RT);
  transpose_colsum_bf16_kernel<<<grid, 256, 0, s>>>((const bf16_t*)src, (bf16_t*)dst, partial, R, C);
  EDL_LAUNCH_CHECK();
  return 0;
}

int edl_transpose_tiles(int R) { return (R + RT - 1) / RT; }

int edl_transpose_bf16_lds(const void* src, void* dst, int R, int C, hipStream_t s) {
  if (R % 8 || C % 8 || R <= 0 || C <= 0) return (int)hipErrorInvalidValue;
  dim3 grid((C + 63) / 64, (R + 63) / 64);
  transpose_bf16_kernel<<<grid, 256, 0, s>>>((const bf16_t*)src, (bf16_t*)dst, R, C);
  EDL_LAUNCH_CHECK();
  return 0;
}

int edl_scale_bf16(void* x, int64_t n, const float* dscale, float hscale, hipStream_t s) {
  if (n % 8) return (int)hipErrorInvalidValue;
  scale_bf16_kernel<<<grid_for(n / 8), 256, 0, s>>>((bf16_t*)x, n / 8, dscale, hscale);
  EDL_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
