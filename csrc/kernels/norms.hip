// RMSNorm and LayerNorm forward/backward (bf16 activations, fp32 math).
//
// Forward: one workgroup per row; each lane keeps its 8-element chunks in
// registers (cols <= 256 lanes x 8 x NC) so the row is read once and written
// once.  Optional fused residual add: s = x + r is written back (the residual
// stream of a pre-norm transformer) and normalised in the same pass.
//
// Backward: a grid of G workgroups sweeps rows; each lane owns fixed columns
// and accumulates dgamma (and dbeta) in registers across its rows, written
// once as a [G, cols] fp32 partial slab; a second small kernel reduces the
// slab column-wise (no float atomics: deterministic, Guideline 12).  The
// residual gradient of the pre-norm block is fused in (dx += dres).
//
// Capability source: SURVEY.md §2.4 N5/N6 (LayerNorm, RMSNorm fwd/bwd).
#include "common.h"

using namespace edl;

namespace {

constexpr int kMaxNC = 4;  // up to 256*8*4 = 8192 columns held in registers

// ---------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------
template <int NC, bool LN>
__global__ __launch_bounds__(256) void norm_fwd_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ res,
                                                       bf16_t* __restrict__ sum_out, const bf16_t* __restrict__ w,
                                                       const bf16_t* __restrict__ b, bf16_t* __restrict__ y,
                                                       float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                       int cols, float eps) {
  __shared__ float red[4];
  const int row = blockIdx.x;
  const int nchunk = cols >> 3;
  const u32x4* xr = reinterpret_cast<const u32x4*>(x + (int64_t)row * cols);
  float v[NC][8];
  float s1 = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int ch = threadIdx.x + c * blockDim.x;
    if (ch < nchunk) {
      unpack8(xr[ch], v[c]);
      if (res) {
        float r[8];
        unpack8(reinterpret_cast<const u32x4*>(res + (int64_t)row * cols)[ch], r);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[c][k] += r[k];
        // round the residual stream to bf16 exactly as stored
        u32x4 sv = pack8(v[c]);
        if (sum_out) reinterpret_cast<u32x4*>(sum_out + (int64_t)row * cols)[ch] = sv;
        unpack8(sv, v[c]);
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) s1 += LN ? v[c][k] : v[c][k] * v[c][k];
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[c][k] = 0.f;
    }
  }
  float mean = 0.f, rstd;
  if (LN) {
    mean = block_sum(s1, red) / cols;
    float s2 = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int ch = threadIdx.x + c * blockDim.x;
      if (ch < nchunk) {
#pragma unroll
        for (int k = 0; k < 8; ++k) { const float d = v[c][k] - mean; s2 += d * d; }
      }
    }
    rstd = rsqrtf(block_sum(s2, red) / cols + eps);
  } else {
    rstd = rsqrtf(block_sum(s1, red) / cols + eps);
  }
  if (threadIdx.x == 0) {
    rstd_out[row] = rstd;
    if (LN) mean_out[row] = mean;
  }
  const u32x4* wr = reinterpret_cast<const u32x4*>(w);
  u32x4* yr = reinterpret_cast<u32x4*>(y + (int64_t)row * cols);
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int ch = threadIdx.x + c * blockDim.x;
    if (ch < nchunk) {
      float wf[8], o[8];
      unpack8(wr[ch], wf);
      if (LN) {
        float bf[8];
        unpack8(reinterpret_cast<const u32x4*>(b)[ch], bf);
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = (v[c][k] - mean) * rstd * wf[k] + bf[k];
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = v[c][k] * rstd * wf[k];
      }
      yr[ch] = pack8(o);
    }
  }
}

// ---------------------------------------------------------------------------
// backward
// ---------------------------------------------------------------------------
// dx = rstd * (dy*w - xhat * mean(dy*w*xhat))                       (RMS)
// dx = rstd * (dy*w - mean(dy*w) - xhat * mean(dy*w*xhat))          (LN)
// partial_w[g][c] = sum_rows dy*xhat ; partial_b[g][c] = sum_rows dy  (LN)
template <int NC, bool LN>
__global__ __launch_bounds__(256) void norm_bwd_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                                       const bf16_t* __restrict__ w, const float* __restrict__ mean_in,
                                                       const float* __restrict__ rstd_in,
                                                       const bf16_t* __restrict__ dres, bf16_t* __restrict__ dx,
                                                       float* __restrict__ pw, float* __restrict__ pb, int rows,
                                                       int cols) {
  __shared__ float red[4];
  const int nchunk = cols >> 3;
  float accw[NC][8], accb[NC][8], wf[NC][8];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int ch = threadIdx.x + c * blockDim.x;
#pragma unroll
    for (int k = 0; k < 8; ++k) { accw[c][k] = 0.f; accb[c][k] = 0.f; wf[c][k] = 0.f; }
    if (ch < nchunk) unpack8(reinterpret_cast<const u32x4*>(w)[ch], wf[c]);
  }
  // Each workgroup sweeps rows with two block reductions per row: the next row's
  // dy / x / dres are loaded into registers before the current row's reductions, so
  // the HBM latency overlaps them (the sweep was latency-bound at ~2-4 TB/s).
  u32x4 nd[NC], nx[NC], nr[NC];
  auto fetch = [&](int r) {
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int ch = threadIdx.x + c * blockDim.x;
      if (ch < nchunk) {
        nd[c] = reinterpret_cast<const u32x4*>(dy + (int64_t)r * cols)[ch];
        nx[c] = reinterpret_cast<const u32x4*>(x + (int64_t)r * cols)[ch];
        if (dres) nr[c] = reinterpret_cast<const u32x4*>(dres + (int64_t)r * cols)[ch];
      }
    }
  };
  if (blockIdx.x < rows) fetch(blockIdx.x);
  for (int row = blockIdx.x; row < rows; row += gridDim.x) {
    u32x4 cd[NC], cx[NC], cr[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) { cd[c] = nd[c]; cx[c] = nx[c]; cr[c] = nr[c]; }
    if (row + (int)gridDim.x < rows) fetch(row + gridDim.x);
    const float rstd = rstd_in[row];
    const float mean = LN ? mean_in[row] : 0.f;
    float xh[NC][8], g[NC][8];
    float s_gx = 0.f, s_g = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int ch = threadIdx.x + c * blockDim.x;
      if (ch < nchunk) {
        float d[8];
        unpack8(cd[c], d);
        unpack8(cx[c], xh[c]);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          xh[c][k] = (xh[c][k] - mean) * rstd;
          g[c][k] = d[k] * wf[c][k];
          s_gx += g[c][k] * xh[c][k];
          if (LN) s_g += g[c][k];
          accw[c][k] += d[k] * xh[c][k];
          if (LN) accb[c][k] += d[k];
        }
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) { xh[c][k] = 0.f; g[c][k] = 0.f; }
      }
    }
    const float m_gx = block_sum(s_gx, red) / cols;
    const float m_g = LN ? block_sum(s_g, red) / cols : 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int ch = threadIdx.x + c * blockDim.x;
      if (ch < nchunk) {
        float o[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = rstd * (g[c][k] - m_g - xh[c][k] * m_gx);
        if (dres) {
          float r[8];
          unpack8(cr[c], r);
#pragma unroll
          for (int k = 0; k < 8; ++k) o[k] += r[k];
        }
        reinterpret_cast<u32x4*>(dx + (int64_t)row * cols)[ch] = pack8(o);
      }
    }
  }
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int ch = threadIdx.x + c * blockDim.x;
    if (ch < nchunk) {
      f32x4* dstw = reinterpret_cast<f32x4*>(pw + (int64_t)blockIdx.x * cols + ch * 8);
      dstw[0] = f32x4{accw[c][0], accw[c][1], accw[c][2], accw[c][3]};
      dstw[1] = f32x4{accw[c][4], accw[c][5], accw[c][6], accw[c][7]};
      if (LN) {
        f32x4* dstb = reinterpret_cast<f32x4*>(pb + (int64_t)blockIdx.x * cols + ch * 8);
        dstb[0] = f32x4{accb[c][0], accb[c][1], accb[c][2], accb[c][3]};
        dstb[1] = f32x4{accb[c][4], accb[c][5], accb[c][6], accb[c][7]};
      }
    }
  }
}

// out[c] (+)= sum_g partial[g][c]; out dtype bf16 (odt=0) or fp32 (odt=1); cols % 4 == 0.
// Column sums of a [G, cols] fp32 partial slab.  A 1024-thread block owns CG column groups
// of 4 (f32x4 loads) and splits the G rows over 1024/CG slices; the slices are summed across
// the lanes of each wave (xor shuffles), then the 16 waves' sums through LDS.  CG is picked
// per call so the launch has >= ~128 blocks: the 16-group block gave BERT-large's 1024-wide
// slabs 16 blocks on 256 CUs (5.5 us per call, 197 calls per step).
template <int CG>
__global__ __launch_bounds__(1024) void colsum_kernel(const float* __restrict__ partial, int G, int cols,
                                                      void* __restrict__ out, int odt, int accumulate) {
  constexpr int SL = 1024 / CG;
  __shared__ f32x4 red[16][CG];
  const int cg = threadIdx.x % CG, sl = threadIdx.x / CG;
  const int c = (blockIdx.x * CG + cg) * 4;
  f32x4 s4[4] = {};
  if (c < cols) {
    int g = sl;
    for (; g + 3 * SL < G; g += 4 * SL) {
#pragma unroll
      for (int u = 0; u < 4; ++u) s4[u] += *reinterpret_cast<const f32x4*>(partial + (int64_t)(g + SL * u) * cols + c);
    }
    for (; g < G; g += SL) s4[0] += *reinterpret_cast<const f32x4*>(partial + (int64_t)g * cols + c);
  }
  f32x4 s = (s4[0] + s4[1]) + (s4[2] + s4[3]);
#pragma unroll
  for (int off = CG; off < 64; off <<= 1) {
#pragma unroll
    for (int k = 0; k < 4; ++k) s[k] += __shfl_xor(s[k], off, 64);
  }
  if ((threadIdx.x & 63) < CG) red[threadIdx.x >> 6][cg] = s;
  __syncthreads();
  if ((int)threadIdx.x >= CG || c >= cols) return;
  s = red[0][cg];
#pragma unroll
  for (int w = 1; w < 16; ++w) s += red[w][cg];
  if (odt == 0) {
    bf16_t* o = reinterpret_cast<bf16_t*>(out) + c;
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = f2bf(accumulate ? s[k] + bf2f(o[k]) : s[k]);
  } else {
    float* o = reinterpret_cast<float*>(out) + c;
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = accumulate ? s[k] + o[k] : s[k];
  }
}

inline int threads_for(int cols) {
  int t = ((cols >> 3) + 63) / 64 * 64;
  if (t > 256) t = 256;
  if (t < 64) t = 64;
  return t;
}

template <bool LN>
int launch_fwd(const bf16_t* x, const bf16_t* res, bf16_t* sum_out, const bf16_t* w, const bf16_t* b, bf16_t* y,
               float* mean, float* rstd, int rows, int cols, float eps, hipStream_t s) {
  if (cols % 8) return (int)hipErrorInvalidValue;
  const int t = threads_for(cols);
  const int nc = ((cols >> 3) + t - 1) / t;
  switch (nc) {
    case 1: norm_fwd_kernel<1, LN><<<rows, t, 0, s>>>(x, res, sum_out, w, b, y, mean, rstd, cols, eps); break;
    case 2: norm_fwd_kernel<2, LN><<<rows, t, 0, s>>>(x, res, sum_out, w, b, y, mean, rstd, cols, eps); break;
    case 3: norm_fwd_kernel<3, LN><<<rows, t, 0, s>>>(x, res, sum_out, w, b, y, mean, rstd, cols, eps); break;
    case 4: norm_fwd_kernel<4, LN><<<rows, t, 0, s>>>(x, res, sum_out, w, b, y, mean, rstd, cols, eps); break;
    default: return (int)hipErrorInvalidValue;
  }
  EDL_LAUNCH_CHECK();
  return 0;
}

template <bool LN>
int launch_bwd(const bf16_t* dy, const bf16_t* x, const bf16_t* w, const float* mean, const float* rstd,
               const bf16_t* dres, bf16_t* dx, float* pw, float* pb, int G, int rows, int cols, hipStream_t s) {
  if (cols % 8) return (int)hipErrorInvalidValue;
  const int t = threads_for(cols);
  const int nc = ((cols >> 3) + t - 1) / t;
  switch (nc) {
    case 1: norm_bwd_kernel<1, LN><<<G, t, 0, s>>>(dy, x, w, mean, rstd, dres, dx, pw, pb, rows, cols); break;
    case 2: norm_bwd_kernel<2, LN><<<G, t, 0, s>>>(dy, x, w, mean, rstd, dres, dx, pw, pb, rows, cols); break;
    case 3: norm_bwd_kernel<3, LN><<<G, t, 0, s>>>(dy, x, w, mean, rstd, dres, dx, pw, pb, rows, cols); break;
    case 4: norm_bwd_kernel<4, LN><<<G, t, 0, s>>>(dy, x, w, mean, rstd, dres, dx, pw, pb, rows, cols); break;
    default: return (int)hipErrorInvalidValue;
  }
  EDL_LAUNCH_CHECK();
  return 0;
}

}  // namespace

extern "C" {

int edl_norm_max_cols() { return 256 * 8 * kMaxNC; }

// Number of row-sweeping workgroups the backward uses (size of the partial slab).
// Sweeping workgroups: 1024 for rows narrower than 4096 (BERT-large d = 1024: 2 waves
// per workgroup, 512 left the sweep latency-bound: 73 -> 40 us), 512 at d >= 4096 where
// the sweep is already 4 waves wide and a bigger [G, cols] slab costs colsum more than
// it saves (profiles/r02_norm_kernels.txt).
int edl_norm_bwd_groups(int rows, int cols) {
  const int g = cols >= 4096 ? 512 : 1024;
  return rows < g ? (rows > 0 ? rows : 1) : g;
}

int edl_rmsnorm_fwd(const void* x, const void* res, void* sum_out, const void* w, void* y, float* rstd, int rows,
                    int cols, float eps, hipStream_t s) {
  return launch_fwd<false>((const bf16_t*)x, (const bf16_t*)res, (bf16_t*)sum_out, (const bf16_t*)w, nullptr,
                           (bf16_t*)y, nullptr, rstd, rows, cols, eps, s);
}

int edl_layernorm_fwd(const void* x, const void* res, void* sum_out, const void* w, const void* b, void* y,
                      float* mean, float* rstd, int rows, int cols, float eps, hipStream_t s) {
  return launch_fwd<true>((const bf16_t*)x, (const bf16_t*)res, (bf16_t*)sum_out, (const bf16_t*)w,
                          (const bf16_t*)b, (bf16_t*)y, mean, rstd, rows, cols, eps, s);
}

// partial_w / partial_b: fp32 [edl_norm_bwd_groups(rows), cols] scratch.
int edl_rmsnorm_bwd(const void* dy, const void* x, const void* w, const float* rstd, const void* dres, void* dx,
                    float* partial_w, int rows, int cols, hipStream_t s) {
  return launch_bwd<false>((const bf16_t*)dy, (const bf16_t*)x, (const bf16_t*)w, nullptr, rstd,
                           (const bf16_t*)dres, (bf16_t*)dx, partial_w, nullptr, edl_norm_bwd_groups(rows, cols), rows,
                           cols, s);
}

int edl_layernorm_bwd(const void* dy, const void* x, const void* w, const float* mean, const float* rstd,
                      const void* dres, void* dx, float* partial_w, float* partial_b, int rows, int cols,
                      hipStream_t s) {
  return launch_bwd<true>((const bf16_t*)dy, (const bf16_t*)x, (const bf16_t*)w, mean, rstd, (const bf16_t*)dres,
                          (bf16_t*)dx, partial_w, partial_b, edl_norm_bwd_groups(rows, cols), rows, cols, s);
}

int edl_colsum(const float* partial, int G, int cols, void* out, int odt, int accumulate, hipStream_t s) {
  if (cols % 4) return (int)hipErrorInvalidValue;
  int cg = 16;   // column groups per block: the widest that still gives >= 128 blocks
  while (cg > 1 && (cols / 4 + cg - 1) / cg < 128) cg >>= 1;
  const unsigned nb = (unsigned)((cols / 4 + cg - 1) / cg);
  switch (cg) {
    case 16: colsum_kernel<16><<<nb, 1024, 0, s>>>(partial, G, cols, out, odt, accumulate); break;
    case 8: colsum_kernel<8><<<nb, 1024, 0, s>>>(partial, G, cols, out, odt, accumulate); break;
    case 4: colsum_kernel<4><<<nb, 1024, 0, s>>>(partial, G, cols, out, odt, accumulate); break;
    case 2: colsum_kernel<2><<<nb, 1024, 0, s>>>(partial, G, cols, out, odt, accumulate); break;
    default: colsum_kernel<1><<<nb, 1024, 0, s>>>(partial, G, cols, out, odt, accumulate); break;
  }
  EDL_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
