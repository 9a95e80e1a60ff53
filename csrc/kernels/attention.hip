// Flash attention forward + backward for gfx950 (bf16, head_dim 128, causal,
// GQA), hand-written on v_mfma_f32_32x32x16_bf16.
//
// Layouts: q [B,S,H,128], k/v [B,S,KV,128] (token-major: exactly what the fused
// RoPE+QKV kernel writes), o / dq like q, dk / dv like k, lse / delta [B,H,S] fp32.
//
// Forward (one workgroup = 4 waves = 128 queries of one head; a wave owns 32
// queries; 64-key K/V tiles double-buffered in LDS):
//   * "swapped" QK^T: S^T = K Q^T, so each lane holds the scores of ONE query
//     (column = lane & 31) for 32 keys; the other 32 keys of the tile are in
//     lane ^ 32 -> the row max/sum need a single cross-half exchange;
//   * online softmax in the exp2 domain; P stays in the accumulator registers
//     and is converted in place to the B operand of O^T += V^T P^T (the
//     accumulator-as-operand identity of cdna_hip_programming.md §3), with the
//     matching permuted key order supplied by ds_read_b64_tr_b16 reads of the
//     row-major V tile;
//   * every LDS tile uses the 256-B-row XOR swizzle that is conflict-free for
//     both ds_read_b128 row reads and transposed reads (guide §5.5 T10 (b)).
// Backward (FA2 split, no float atomics):
//   * dK/dV kernel: a workgroup owns 128 keys of one KV head (a wave 32 keys,
//     K/V rows in registers, dK^T/dV^T accumulators resident for the whole
//     sweep) and sweeps every query head of the GQA group x 32-query slices
//     (Q/dO slices double-buffered in LDS);
//   * dQ kernel: the forward's structure with dP^T = V dO^T and dQ^T += K^T dS^T.
// Capability source: Llama-3 training workloads (BASELINE.json configs 3/5).
#include "common.h"

using namespace edl;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef short i16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) i16x4 lds_i16x4;

constexpr int HD = 128;        // head dim
constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

// byte offset of 16-B chunk c of row r in a [rows][256 B] LDS tile
__device__ __forceinline__ int swz(int r, int c) {
  return (r << 8) + ((c ^ (((r & 3) << 2) | ((r >> 2) & 3))) << 4);
}

__device__ __forceinline__ f32x16 mfma(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// A/B operand "row read": 8 bf16 of row r, k-step s (16 elements), lane half h
__device__ __forceinline__ bf16x8 row_read(const char* tile, int r, int s, int h) {
  return *reinterpret_cast<const bf16x8*>(tile + swz(r, 2 * s + h));
}

// A operand with rows = d (32*dt + lane&31) and k = rows kb.. of a row-major
// [k][d] tile in the permuted order of an accumulator-as-B operand:
// element j <-> k row kb + 8*(j>>2) + (j&3).
__device__ __forceinline__ bf16x8 tr_read(const char* tile, int kb, int dt, int lane) {
  const int i = lane & 15, qq = i >> 2, p = i & 3;
  const int col = dt * 32 + ((lane >> 4) & 1) * 16 + 4 * p;
  const int c = col >> 3, half = (col >> 2) & 1;
  const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(tile + swz(kb + qq, c) + half * 8));
  const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(tile + swz(kb + 8 + qq, c) + half * 8));
  const i16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

// accumulator registers 8*s2 .. 8*s2+7 -> bf16 B operand
__device__ __forceinline__ bf16x8 acc_to_b(const f32x16& acc, int s2) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)acc[8 * s2 + j];
  return r;
}

// row (within a 32-row tile) of accumulator register i for lane half h
__device__ __forceinline__ int acc_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

// stage `rows` x 256 B of a token-major tensor into a swizzled LDS tile
template <int ROWS>
__device__ __forceinline__ void load_rows(u32x4 (&regs)[ROWS / 16], const bf16_t* base, int64_t stride, int row0,
                                          int S) {
#pragma unroll
  for (int i = 0; i < ROWS / 16; ++i) {
    const int idx = threadIdx.x + 256 * i;
    const int r = idx >> 4, c = idx & 15;
    const int row = row0 + r;
    regs[i] = row < S ? *reinterpret_cast<const u32x4*>(base + (int64_t)row * stride + c * 8) : u32x4{0, 0, 0, 0};
  }
}
template <int ROWS>
__device__ __forceinline__ void store_rows(char* tile, const u32x4 (&regs)[ROWS / 16]) {
#pragma unroll
  for (int i = 0; i < ROWS / 16; ++i) {
    const int idx = threadIdx.x + 256 * i;
    *reinterpret_cast<u32x4*>(tile + swz(idx >> 4, idx & 15)) = regs[i];
  }
}

__device__ __forceinline__ bf16x8 load_frag(const bf16_t* rowp, int s, int h, bool valid) {
  if (!valid) return bf16x8{};
  return *reinterpret_cast<const bf16x8*>(rowp + (2 * s + h) * 8);
}

// write an O^T-style accumulator set (rows d, col = this lane's token) as 4-element runs
__device__ __forceinline__ void store_accT(bf16_t* rowp, const f32x16 (&acc)[4], float mul, int h) {
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      u32x2 w;
      w[0] = pack2(acc[dt][4 * g] * mul, acc[dt][4 * g + 1] * mul);
      w[1] = pack2(acc[dt][4 * g + 2] * mul, acc[dt][4 * g + 3] * mul);
      *reinterpret_cast<u32x2*>(rowp + dt * 32 + 8 * g + 4 * h) = w;
    }
  }
}

// ---------------------------------------------------------------------------
// forward: a wave owns QG*32 queries (QG column groups); every K / V fragment
// read from LDS feeds QG MFMAs.
// ---------------------------------------------------------------------------
template <bool CAUSAL, int QG>
__global__ __launch_bounds__(256, QG == 1 ? 2 : 1) void attn_fwd_kernel(const bf16_t* __restrict__ q, const bf16_t* __restrict__ k,
                                                          const bf16_t* __restrict__ v, bf16_t* __restrict__ o,
                                                          float* __restrict__ lse, int S, int H, int KV,
                                                          float scale_log2) {
  constexpr int BQ = 128 * QG;
  __shared__ __attribute__((aligned(16))) char smem[2 * 32768];
  const int qb = gridDim.x - 1 - blockIdx.x;  // longest causal rows first
  const int hq = blockIdx.y, b = blockIdx.z, hk = hq / (H / KV);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, l31 = lane & 31;
  const int q0 = qb * BQ;
  const int wq0 = q0 + 32 * QG * w;  // first query of this wave
  const int64_t qs = (int64_t)H * HD, ks = (int64_t)KV * HD;
  const bf16_t* qp = q + (int64_t)b * S * qs + hq * HD;
  const bf16_t* kp = k + (int64_t)b * S * ks + hk * HD;
  const bf16_t* vp = v + (int64_t)b * S * ks + hk * HD;

  bf16x8 qf[QG][8];
#pragma unroll
  for (int g = 0; g < QG; ++g) {
    const int qr = wq0 + 32 * g + l31;
#pragma unroll
    for (int s = 0; s < 8; ++s) qf[g][s] = load_frag(qp + (int64_t)qr * qs, s, h, qr < S);
  }
  const int kv_end = CAUSAL ? min(S, q0 + BQ) : S;
  const int ntiles = (kv_end + 63) / 64;
  f32x16 oacc[QG][4];
  float m[QG], lsum[QG];
#pragma unroll
  for (int g = 0; g < QG; ++g) {
    m[g] = -1e30f;
    lsum[g] = 0.f;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) oacc[g][dt] = f32x16{};
  }

  u32x4 kreg[4], vreg[4];
  load_rows<64>(kreg, kp, ks, 0, S);
  load_rows<64>(vreg, vp, ks, 0, S);
  store_rows<64>(smem, kreg);
  store_rows<64>(smem + 16384, vreg);
  __syncthreads();

  for (int it = 0; it < ntiles; ++it) {
    const int kv0 = it * 64;
    if (it + 1 < ntiles) {
      load_rows<64>(kreg, kp, ks, kv0 + 64, S);
      load_rows<64>(vreg, vp, ks, kv0 + 64, S);
    }
    const char* Ks = smem + (it & 1) * 32768;
    const char* Vs = Ks + 16384;
    const bool wave_visible = !CAUSAL || kv0 <= wq0 + 32 * QG - 1;
    if (wave_visible) {
      f32x16 sacc[QG][2];
#pragma unroll
      for (int g = 0; g < QG; ++g) sacc[g][0] = sacc[g][1] = f32x16{};
#pragma unroll
      for (int t = 0; t < 2; ++t) {
#pragma unroll
        for (int s = 0; s < 8; ++s) {
          const bf16x8 a = row_read(Ks, 32 * t + l31, s, h);
#pragma unroll
          for (int g = 0; g < QG; ++g) sacc[g][t] = mfma(a, qf[g][s], sacc[g][t]);
        }
      }
      const bool need_mask = (kv0 + 64 > S) || (CAUSAL && kv0 + 63 > wq0);
      bool grow = false;
      float alpha[QG];
#pragma unroll
      for (int g = 0; g < QG; ++g) {
        const int qr = wq0 + 32 * g + l31;
        float mx = -1e30f;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            float x = sacc[g][t][i] * scale_log2;
            if (need_mask) {
              const int key = kv0 + 32 * t + acc_row(i, h);
              if (key >= S || (CAUSAL && key > qr)) x = -INFINITY;
            }
            sacc[g][t][i] = x;
            mx = fmaxf(mx, x);
          }
        }
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        const float mnew = fmaxf(m[g], mx);
        grow |= mnew > m[g];
        alpha[g] = exp2f(m[g] - mnew);
        m[g] = mnew;
        float ps = 0.f;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const float p = exp2f(sacc[g][t][i] - mnew);
            sacc[g][t][i] = p;
            ps += p;
          }
        }
        lsum[g] = lsum[g] * alpha[g] + ps;
      }
      // exact lazy rescale: only when some row max of this wave grew
      if (__any(grow)) {
#pragma unroll
        for (int g = 0; g < QG; ++g) {
#pragma unroll
          for (int dt = 0; dt < 4; ++dt) oacc[g][dt] *= alpha[g];
        }
      }
#pragma unroll
      for (int t = 0; t < 2; ++t) {
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          bf16x8 pb[QG];
#pragma unroll
          for (int g = 0; g < QG; ++g) pb[g] = acc_to_b(sacc[g][t], s2);
#pragma unroll
          for (int dt = 0; dt < 4; ++dt) {
            const bf16x8 a = tr_read(Vs, 32 * t + 16 * s2 + 4 * h, dt, lane);
#pragma unroll
            for (int g = 0; g < QG; ++g) oacc[g][dt] = mfma(a, pb[g], oacc[g][dt]);
          }
        }
      }
    }
    __syncthreads();
    if (it + 1 < ntiles) {
      char* nxt = smem + ((it + 1) & 1) * 32768;
      store_rows<64>(nxt, kreg);
      store_rows<64>(nxt + 16384, vreg);
    }
    __syncthreads();
  }
#pragma unroll
  for (int g = 0; g < QG; ++g) {
    const int qr = wq0 + 32 * g + l31;
    const float ltot = lsum[g] + __shfl_xor(lsum[g], 32, 64);
    if (qr < S) {
      store_accT(o + (int64_t)b * S * qs + (int64_t)qr * qs + hq * HD, oacc[g], 1.f / ltot, h);
      if (h == 0) lse[((int64_t)b * H + hq) * S + qr] = (m[g] + log2f(ltot)) * LN2;
    }
  }
}

// ---------------------------------------------------------------------------
// backward preprocess: delta = rowsum(dO * O)   (16 lanes per row, 16 B each)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void attn_bwd_delta_kernel(const bf16_t* __restrict__ o,
                                                             const bf16_t* __restrict__ dout,
                                                             float* __restrict__ delta, int S, int H,
                                                             int64_t nrows) {
  const int64_t row = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 4;  // row = (b*S + s)*H + h
  const int c = threadIdx.x & 15;
  float acc = 0.f;
  if (row < nrows) {
    float a[8], d[8];
    unpack8(reinterpret_cast<const u32x4*>(o + row * HD)[c], a);
    unpack8(reinterpret_cast<const u32x4*>(dout + row * HD)[c], d);
#pragma unroll
    for (int i = 0; i < 8; ++i) acc += a[i] * d[i];
  }
#pragma unroll
  for (int off = 8; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 16);
  if (c == 0 && row < nrows) {
    const int64_t hh = row % H, tok = row / H, s = tok % S, b = tok / S;
    delta[(b * H + hh) * S + s] = acc;
  }
}

// ---------------------------------------------------------------------------
// backward: dK, dV.  A workgroup owns 128 keys of one KV head (a wave 32 keys,
// K/V in registers, dK^T/dV^T accumulators resident) and sweeps 64-query
// tiles (two 32-row sub-slices) of every query head of the GQA group.
// ---------------------------------------------------------------------------
template <bool CAUSAL>
__global__ __launch_bounds__(256, 1) void attn_bwd_dkdv_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    const bf16_t* __restrict__ dout, const float* __restrict__ lse, const float* __restrict__ delta,
    bf16_t* __restrict__ dk, bf16_t* __restrict__ dv, int S, int H, int KV, float scale_log2, float scale) {
  constexpr int QT = 64;  // queries per staged tile
  // 2 stages x (Q tile 16 KB + dO tile 16 KB) + 2 x (lse2, delta) x 64 floats
  __shared__ __attribute__((aligned(16))) char smem[2 * 32768 + 2 * 512];
  const int kb = blockIdx.x, hk = blockIdx.y, b = blockIdx.z;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, l31 = lane & 31;
  const int group = H / KV;
  const int64_t qs = (int64_t)H * HD, ks = (int64_t)KV * HD;
  const int mykey = kb * 128 + 32 * w + l31;
  const bf16_t* krow = k + (int64_t)b * S * ks + (int64_t)mykey * ks + hk * HD;
  const bf16_t* vrow = v + (int64_t)b * S * ks + (int64_t)mykey * ks + hk * HD;
  bf16x8 kf[8], vf[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    kf[s] = load_frag(krow, s, h, mykey < S);
    vf[s] = load_frag(vrow, s, h, mykey < S);
  }
  f32x16 dka[4], dva[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    dka[dt] = f32x16{};
    dva[dt] = f32x16{};
  }
  const int nqt = (S + QT - 1) / QT;
  const int qt0 = CAUSAL ? (kb * 128) / QT : 0;
  const int per_head = nqt - qt0;
  const int total = per_head * group;
  const int wave_key_lo = kb * 128 + 32 * w;

  u32x4 qreg[4], dreg[4];
  float lreg = 0.f, dlreg = 0.f;
  auto fetch = [&](int j) {
    const int hq = hk * group + j / per_head;
    const int q0 = (qt0 + j % per_head) * QT;
    load_rows<QT>(qreg, q + (int64_t)b * S * qs + hq * HD, qs, q0, S);
    load_rows<QT>(dreg, dout + (int64_t)b * S * qs + hq * HD, qs, q0, S);
    if (threadIdx.x < QT) {
      const int qq = q0 + threadIdx.x;
      lreg = qq < S ? lse[((int64_t)b * H + hq) * S + qq] * LOG2E : 0.f;
      dlreg = qq < S ? delta[((int64_t)b * H + hq) * S + qq] : 0.f;
    }
  };
  auto commit = [&](int st) {
    char* base = smem + st * 32768;
    store_rows<QT>(base, qreg);
    store_rows<QT>(base + 16384, dreg);
    if (threadIdx.x < QT) {
      float* lf = reinterpret_cast<float*>(smem + 2 * 32768 + st * 512);
      lf[threadIdx.x] = lreg;
      lf[QT + threadIdx.x] = dlreg;
    }
  };
  if (total > 0) {
    fetch(0);
    commit(0);
  }
  __syncthreads();
  for (int j = 0; j < total; ++j) {
    if (j + 1 < total) fetch(j + 1);
    const int st = j & 1;
    const char* Qs = smem + st * 32768;
    const char* Ds = Qs + 16384;
    const float* L2 = reinterpret_cast<const float*>(smem + 2 * 32768 + st * 512);
    const int q0 = (qt0 + j % per_head) * QT;
#pragma unroll
    for (int sub = 0; sub < QT / 32; ++sub) {
      const int qs0 = q0 + 32 * sub;
      if (CAUSAL && qs0 + 31 < wave_key_lo) continue;  // wave-uniform: all masked
      const int rb = 32 * sub;  // row base inside the staged tile
      f32x16 sa = f32x16{};
#pragma unroll
      for (int s = 0; s < 8; ++s) sa = mfma(row_read(Qs, rb + l31, s, h), kf[s], sa);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int r = acc_row(i, h);
        const int qi = qs0 + r;
        float p = exp2f(sa[i] * scale_log2 - L2[rb + r]);
        if (qi >= S || mykey >= S || (CAUSAL && mykey > qi)) p = 0.f;
        sa[i] = p;
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8 pb = acc_to_b(sa, s2);
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) dva[dt] = mfma(tr_read(Ds, rb + 16 * s2 + 4 * h, dt, lane), pb, dva[dt]);
      }
      f32x16 dp = f32x16{};
#pragma unroll
      for (int s = 0; s < 8; ++s) dp = mfma(row_read(Ds, rb + l31, s, h), vf[s], dp);
#pragma unroll
      for (int i = 0; i < 16; ++i) dp[i] = sa[i] * (dp[i] - L2[QT + rb + acc_row(i, h)]);
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8 db = acc_to_b(dp, s2);
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) dka[dt] = mfma(tr_read(Qs, rb + 16 * s2 + 4 * h, dt, lane), db, dka[dt]);
      }
    }
    __syncthreads();
    if (j + 1 < total) commit((j + 1) & 1);
    __syncthreads();
  }
  if (mykey < S) {
    store_accT(dk + (int64_t)b * S * ks + (int64_t)mykey * ks + hk * HD, dka, scale, h);
    store_accT(dv + (int64_t)b * S * ks + (int64_t)mykey * ks + hk * HD, dva, 1.f, h);
  }
}

// ---------------------------------------------------------------------------
// backward: dQ (a wave owns QG*32 queries; K/V fragments feed QG MFMAs)
// ---------------------------------------------------------------------------
template <bool CAUSAL, int QG>
__global__ __launch_bounds__(256, QG == 1 ? 2 : 1) void attn_bwd_dq_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    const bf16_t* __restrict__ dout, const float* __restrict__ lse, const float* __restrict__ delta,
    bf16_t* __restrict__ dq, int S, int H, int KV, float scale_log2, float scale) {
  constexpr int BQ = 128 * QG;
  __shared__ __attribute__((aligned(16))) char smem[2 * 32768];
  const int qb = gridDim.x - 1 - blockIdx.x;
  const int hq = blockIdx.y, b = blockIdx.z, hk = hq / (H / KV);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, l31 = lane & 31;
  const int q0 = qb * BQ;
  const int wq0 = q0 + 32 * QG * w;
  const int64_t qs = (int64_t)H * HD, ks = (int64_t)KV * HD;
  const bf16_t* kp = k + (int64_t)b * S * ks + hk * HD;
  const bf16_t* vp = v + (int64_t)b * S * ks + hk * HD;
  bf16x8 qf[QG][8], df[QG][8];
  float l2[QG], dl[QG];
  f32x16 dqa[QG][4];
#pragma unroll
  for (int g = 0; g < QG; ++g) {
    const int qr = wq0 + 32 * g + l31;
    const bf16_t* qrow = q + (int64_t)b * S * qs + (int64_t)qr * qs + hq * HD;
    const bf16_t* drow = dout + (int64_t)b * S * qs + (int64_t)qr * qs + hq * HD;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      qf[g][s] = load_frag(qrow, s, h, qr < S);
      df[g][s] = load_frag(drow, s, h, qr < S);
    }
    l2[g] = qr < S ? lse[((int64_t)b * H + hq) * S + qr] * LOG2E : 0.f;
    dl[g] = qr < S ? delta[((int64_t)b * H + hq) * S + qr] : 0.f;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dqa[g][dt] = f32x16{};
  }
  const int kv_end = CAUSAL ? min(S, q0 + BQ) : S;
  const int ntiles = (kv_end + 63) / 64;
  u32x4 kreg[4], vreg[4];
  load_rows<64>(kreg, kp, ks, 0, S);
  load_rows<64>(vreg, vp, ks, 0, S);
  store_rows<64>(smem, kreg);
  store_rows<64>(smem + 16384, vreg);
  __syncthreads();
  for (int it = 0; it < ntiles; ++it) {
    const int kv0 = it * 64;
    if (it + 1 < ntiles) {
      load_rows<64>(kreg, kp, ks, kv0 + 64, S);
      load_rows<64>(vreg, vp, ks, kv0 + 64, S);
    }
    const char* Ks = smem + (it & 1) * 32768;
    const char* Vs = Ks + 16384;
    const bool visible = !(CAUSAL && kv0 > wq0 + 32 * QG - 1);
    if (visible) {
      const bool need_mask = (kv0 + 64 > S) || (CAUSAL && kv0 + 63 > wq0);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        f32x16 st[QG], dpt[QG];
#pragma unroll
        for (int g = 0; g < QG; ++g) st[g] = dpt[g] = f32x16{};
#pragma unroll
        for (int s = 0; s < 8; ++s) {
          const bf16x8 a = row_read(Ks, 32 * t + l31, s, h);
#pragma unroll
          for (int g = 0; g < QG; ++g) st[g] = mfma(a, qf[g][s], st[g]);
        }
#pragma unroll
        for (int s = 0; s < 8; ++s) {
          const bf16x8 a = row_read(Vs, 32 * t + l31, s, h);
#pragma unroll
          for (int g = 0; g < QG; ++g) dpt[g] = mfma(a, df[g][s], dpt[g]);
        }
#pragma unroll
        for (int g = 0; g < QG; ++g) {
          const int qr = wq0 + 32 * g + l31;
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            float p = exp2f(st[g][i] * scale_log2 - l2[g]);
            if (need_mask) {
              const int key = kv0 + 32 * t + acc_row(i, h);
              if (key >= S || (CAUSAL && key > qr)) p = 0.f;
            }
            dpt[g][i] = p * (dpt[g][i] - dl[g]);  // dS^T
          }
        }
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          bf16x8 db[QG];
#pragma unroll
          for (int g = 0; g < QG; ++g) db[g] = acc_to_b(dpt[g], s2);
#pragma unroll
          for (int dt = 0; dt < 4; ++dt) {
            const bf16x8 a = tr_read(Ks, 32 * t + 16 * s2 + 4 * h, dt, lane);
#pragma unroll
            for (int g = 0; g < QG; ++g) dqa[g][dt] = mfma(a, db[g], dqa[g][dt]);
          }
        }
      }
    }
    __syncthreads();
    if (it + 1 < ntiles) {
      char* nxt = smem + ((it + 1) & 1) * 32768;
      store_rows<64>(nxt, kreg);
      store_rows<64>(nxt + 16384, vreg);
    }
    __syncthreads();
  }
#pragma unroll
  for (int g = 0; g < QG; ++g) {
    const int qr = wq0 + 32 * g + l31;
    if (qr < S) store_accT(dq + (int64_t)b * S * qs + (int64_t)qr * qs + hq * HD, dqa[g], scale, h);
  }
}

}  // namespace

extern "C" {

int edl_attn_fwd(const void* q, const void* k, const void* v, void* o, float* lse, int B, int S, int H, int KV,
                 int D, int causal, float scale, hipStream_t s) {
  if (D != HD || H % KV != 0 || S <= 0) return (int)hipErrorInvalidValue;
  // QG = 2 (64 rows per wave) halves LDS bytes per MFMA but needs 512 registers
  // -> 1 wave/SIMD, which measured 2.7x slower (latency exposed); keep QG = 1.
  constexpr int QG = 1;
  dim3 grid((S + 128 * QG - 1) / (128 * QG), H, B);
  const float sl2 = scale * LOG2E;
  if (causal)
    attn_fwd_kernel<true, QG><<<grid, 256, 0, s>>>((const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v,
                                                   (bf16_t*)o, lse, S, H, KV, sl2);
  else
    attn_fwd_kernel<false, QG><<<grid, 256, 0, s>>>((const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v,
                                                    (bf16_t*)o, lse, S, H, KV, sl2);
  EDL_LAUNCH_CHECK();
  return 0;
}

// delta: fp32 [B,H,S] scratch filled here.
int edl_attn_bwd(const void* q, const void* k, const void* v, const void* o, const void* dout, const float* lse,
                 float* delta, void* dq, void* dk, void* dv, int B, int S, int H, int KV, int D, int causal,
                 float scale, hipStream_t s) {
  if (D != HD || H % KV != 0 || S <= 0) return (int)hipErrorInvalidValue;
  const int64_t nrows = (int64_t)B * S * H;
  attn_bwd_delta_kernel<<<(unsigned)((nrows * 16 + 255) / 256), 256, 0, s>>>((const bf16_t*)o, (const bf16_t*)dout,
                                                                            delta, S, H, nrows);
  EDL_LAUNCH_CHECK();
  const float sl2 = scale * LOG2E;
  constexpr int QG = 1;
  dim3 gkv((S + 127) / 128, KV, B), gq((S + 128 * QG - 1) / (128 * QG), H, B);
  if (causal) {
    attn_bwd_dkdv_kernel<true><<<gkv, 256, 0, s>>>((const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v,
                                                   (const bf16_t*)dout, lse, delta, (bf16_t*)dk, (bf16_t*)dv, S, H,
                                                   KV, sl2, scale);
    EDL_LAUNCH_CHECK();
    attn_bwd_dq_kernel<true, QG><<<gq, 256, 0, s>>>((const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v,
                                                (const bf16_t*)dout, lse, delta, (bf16_t*)dq, S, H, KV, sl2, scale);
  } else {
    attn_bwd_dkdv_kernel<false><<<gkv, 256, 0, s>>>((const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v,
                                                    (const bf16_t*)dout, lse, delta, (bf16_t*)dk, (bf16_t*)dv, S, H,
                                                    KV, sl2, scale);
    EDL_LAUNCH_CHECK();
    attn_bwd_dq_kernel<false, QG><<<gq, 256, 0, s>>>((const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v,
                                                 (const bf16_t*)dout, lse, delta, (bf16_t*)dq, S, H, KV, sl2, scale);
  }
  EDL_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
