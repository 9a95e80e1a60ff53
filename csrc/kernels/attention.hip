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
#include <cstdlib>
#include <type_traits>

#include "common.h"

using namespace edl;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef short i16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) i16x4 lds_i16x4;
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(3))) char lds_char;
typedef __attribute__((address_space(3))) const bf16x8 lds_bf16x8;

constexpr int HD = 128;        // head dim
constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

// byte offset of 16-B chunk c of row r in a [rows][2*D B] LDS tile.  D = 128: 256-B
// rows, XOR-swizzled so the 32x32x16 fragments' ds_read_b128 row reads and
// ds_read_b64_tr_b16 transposed reads are both conflict-free (guide §5.5 T10 (b)).
// D = 64: 128-B rows, two per 256-B bank window; x(r) = ((r>>2)&3) | (((r>>1)&1)<<2)
// gives every 16-lane b128 pass (rows l&31 of one chunk) and every 32-lane tr_b16
// pass (4 rows x 4 chunks) 16 distinct 16-B bank groups (MI355X_MICROARCH.md LDS table).
template <int D>
__device__ __forceinline__ int swzd(int r, int c) {
  if constexpr (D == 128)
    return (r << 8) + ((c ^ (((r & 3) << 2) | ((r >> 2) & 3))) << 4);
  else
    return (r << 7) + ((c ^ (((r >> 2) & 3) | (((r >> 1) & 1) << 2))) << 4);
}
template <int D>
__device__ __forceinline__ int swz_x(int r) {   // the XOR of row r (LDS-DMA lane -> chunk)
  if constexpr (D == 128)
    return ((r & 3) << 2) | ((r >> 2) & 3);
  else
    return ((r >> 2) & 3) | (((r >> 1) & 1) << 2);
}
__device__ __forceinline__ int swz(int r, int c) { return swzd<128>(r, c); }

__device__ __forceinline__ f32x16 mfma(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// A/B operand "row read": 8 bf16 of row r, k-step s (16 elements), lane half h
template <int D = 128>
__device__ __forceinline__ bf16x8 row_read(const char* tile, int r, int s, int h) {
  return *reinterpret_cast<const bf16x8*>(tile + swzd<D>(r, 2 * s + h));
}

// A operand with rows = d (32*dt + lane&31) and k = rows kb.. of a row-major
// [k][d] tile in the permuted order of an accumulator-as-B operand:
// element j <-> k row kb + 8*(j>>2) + (j&3).
template <int D = 128>
__device__ __forceinline__ bf16x8 tr_read(const char* tile, int kb, int dt, int lane) {
  const int i = lane & 15, qq = i >> 2, p = i & 3;
  const int col = dt * 32 + ((lane >> 4) & 1) * 16 + 4 * p;
  const int c = col >> 3, half = (col >> 2) & 1;
  const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(tile + swzd<D>(kb + qq, c) + half * 8));
  const i16x4 hi =
      __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(tile + swzd<D>(kb + 8 + qq, c) + half * 8));
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

// Work decode of the (query block, query head, batch) grids of the forward and dQ
// kernels.  xcd = 0: blockIdx as launched (query block reversed: longest causal rows
// first).  xcd = 1 (needs B*KV % 8 == 0): workgroups are dealt round-robin over the 8
// XCDs (blocks b and b+8 share one, MI355X_MICROARCH.md 'Workgroup dispatch'), so block
// b is given K/V group (b % 8) + 8 j: every XCD serves whole GQA groups and one group's
// K and V (4 MiB at S = 8192) stay in that XCD's L2 instead of all groups thrashing
// every L2; query blocks still run longest first within each XCD.
__device__ __forceinline__ void grid_decode(int xcd, int H, int KV, int& qb, int& hq, int& b) {
  if (!xcd) {
    qb = gridDim.x - 1 - blockIdx.x;
    hq = blockIdx.y;
    b = blockIdx.z;
    return;
  }
  const int id = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  const int gsz = H / KV, per = (int)gridDim.z * KV / 8;   // q heads per group, groups per XCD
  const int slot = id >> 3, rank = slot / (per * gsz), rem = slot % (per * gsz);
  const int g = (id & 7) + 8 * (rem / gsz);
  qb = gridDim.x - 1 - rank;
  b = g / KV;
  hq = (g % KV) * gsz + rem % gsz;
}

// v_exp_f32 directly (exp2f() adds a denormal range fix-up: 3 extra VALU per call)
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// reductions across the two 32-lane halves with v_permlane32_swap (no LDS traffic)
__device__ __forceinline__ float xhalf_max(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xhalf_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// stage `rows` x 256 B of a token-major tensor into a swizzled LDS tile.  Rows
// past the end are clamped to the last row (no exec-mask branches in the hot
// loop); the score mask / zero probabilities make their contribution vanish.
template <int ROWS>
__device__ __forceinline__ void load_rows(u32x4 (&regs)[ROWS / 16], const bf16_t* base, int64_t stride, int row0,
                                          int S) {
#pragma unroll
  for (int i = 0; i < ROWS / 16; ++i) {
    const int idx = threadIdx.x + 256 * i;
    const int r = idx >> 4, c = idx & 15;
    const int row = min(row0 + r, S - 1);
    regs[i] = *reinterpret_cast<const u32x4*>(base + (int64_t)row * stride + c * 8);
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

// 8 bf16 of a (clamped, always valid) row pointer: k-step s, lane half h
// LDS-DMA staging: fill ROWS x 256 B of a swizzled LDS tile straight from
// global memory with buffer_load_dwordx4 ... lds (no staging registers, no
// ds_write).  Each wave-instruction writes one contiguous 1-KiB piece = 4 rows,
// lane l landing at piece + 16*l, so lane l fetches the chunk that the XOR
// swizzle maps to that slot.  The per-lane byte offsets are loop-invariant
// (PER_WAVE VGPRs); the tile's first row goes in the scalar offset.  The buffer
// descriptor's range ends at row S of this (batch, head) slice, so rows past
// the end read as zeros (and are masked).  Completion: vmcnt + barrier.
typedef __amdgpu_buffer_rsrc_t rsrc_t;

__device__ __forceinline__ rsrc_t make_rsrc(const void* base, int64_t nbytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)nbytes, 0x00020000);
}

// The LDS-DMA builtin exists only for the device target; clang's host pass
// instantiates kernel templates too, and an (otherwise silent) deferred error
// there drops the kernels' host launch stubs -> keep it out of the host pass.
__device__ __forceinline__ void buffer_load_lds16(rsrc_t rs, void* lds, uint32_t voff, uint32_t soff) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)lds, 16, voff, soff, 0, 0);
#endif
}
__device__ __forceinline__ void buffer_load_lds4(rsrc_t rs, void* lds, uint32_t voff, uint32_t soff) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)lds, 4, voff, soff, 0, 0);
#endif
}

template <int ROWS, int NWAVES, int D = 128>
struct DmaPlan {
  static constexpr int LPR = D / 8;                  // lanes (16-B chunks) per row
  static constexpr int RPP = 64 / LPR;               // rows per 1-KiB piece
  static constexpr int PER_WAVE = ROWS / RPP / NWAVES;
  uint32_t voff[PER_WAVE];
  __device__ __forceinline__ DmaPlan(int64_t stride_elems, int w, int lane) {
#pragma unroll
    for (int i = 0; i < PER_WAVE; ++i) {
      const int r = RPP * (w * PER_WAVE + i) + lane / LPR;
      const int c = (lane % LPR) ^ swz_x<D>(r);
      voff[i] = (uint32_t)((r * stride_elems + c * 8) * 2);
    }
  }
  // rows row0 .. row0+ROWS-1 (row0 * row_bytes goes in the scalar offset)
  __device__ __forceinline__ void issue(char* tile, rsrc_t rs, uint32_t soff, int w) const {
#pragma unroll
    for (int i = 0; i < PER_WAVE; ++i)
      buffer_load_lds16(rs, tile + (w * PER_WAVE + i) * 1024, voff[i], soff);
  }
};

// 64 consecutive fp32 -> LDS, one wave-instruction (past-the-end reads as 0)
__device__ __forceinline__ void dma_f32x64(float* dst, rsrc_t rs, int i0, int lane) {
  buffer_load_lds4(rs, dst, (uint32_t)lane * 4, (uint32_t)i0 * 4);
}

// all of this wave's outstanding vector-memory ops (incl. LDS-DMA) done
__device__ __forceinline__ void wait_vm() { __builtin_amdgcn_s_waitcnt(0x0F70); }

__device__ __forceinline__ bf16x8 load_frag(const bf16_t* rowp, int s, int h) {
  return *reinterpret_cast<const bf16x8*>(rowp + (2 * s + h) * 8);
}

// write an O^T-style accumulator set (rows d, col = this lane's token) as 4-element runs
template <int ND>
__device__ __forceinline__ void store_accT(bf16_t* rowp, const f32x16 (&acc)[ND], float mul, int h) {
#pragma unroll
  for (int dt = 0; dt < ND; ++dt) {
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
// forward: a wave owns 32 queries; one 64-key tile = 16 MFMAs for S^T and 16
// for O^T.  The per-tile VALU work is kept to ~4 instructions per score
// (max3, fma+exp, add, half a cvt_pk): masks only on the diagonal / tail tile.
// ---------------------------------------------------------------------------
template <bool MASK, bool CAUSAL, int D>
__device__ __forceinline__ void fwd_tile(const char* Ks, const char* Vs, const bf16x8 (&qf)[D / 16],
                                         f32x16 (&oacc)[D / 32], float& m, float& lsum, int kv0, int qr, int S,
                                         float sl2, int lane) {
  const int h = lane >> 5, l31 = lane & 31;
  f32x16 sacc[2];
  sacc[0] = sacc[1] = f32x16{};
#pragma unroll
  for (int t = 0; t < 2; ++t) {
#pragma unroll
    for (int s = 0; s < D / 16; ++s) sacc[t] = mfma(row_read<D>(Ks, 32 * t + l31, s, h), qf[s], sacc[t]);
  }
  if (MASK) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int key = kv0 + 32 * t + acc_row(i, h);
        if (key >= S || (CAUSAL && key > qr)) sacc[t][i] = -INFINITY;
      }
    }
  }
  float mx = sacc[0][0];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
#pragma unroll
    for (int i = 0; i < 16; ++i) mx = fmaxf(mx, sacc[t][i]);
  }
  mx = xhalf_max(mx);
  // Running max in the scaled log2 domain (sl2 > 0 commutes with max).  Thresholded
  // lazy rescale: the reference max m only moves when some row of the wave grew by
  // more than 2^8; otherwise p = exp2(s - m) <= 256 is used as is (fp32 sums, bf16 P
  // keeps its 8 exponent bits), and O, l stay consistent with the stale m.  This
  // skips the 64-register O rescale on almost every tile after the first few.
  const float mxs = mx * sl2;
  if (__any(mxs > m + 8.f)) {
    const float mnew = fmaxf(m, mxs);
    const float alpha = fast_exp2(m - mnew);
    m = mnew;
    lsum *= alpha;
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt) oacc[dt] *= alpha;
  }
  const float negm = -m;
  float ps = 0.f;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float p = fast_exp2(__builtin_fmaf(sacc[t][i], sl2, negm));
      sacc[t][i] = p;
      ps += p;
    }
  }
  lsum += ps;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const bf16x8 pb = acc_to_b(sacc[t], s2);
#pragma unroll
      for (int dt = 0; dt < D / 32; ++dt)
        oacc[dt] = mfma(tr_read<D>(Vs, 32 * t + 16 * s2 + 4 * h, dt, lane), pb, oacc[dt]);
    }
  }
}

template <bool CAUSAL, int D>
__global__ __launch_bounds__(256, 2) void attn_fwd_kernel(const bf16_t* __restrict__ q, const bf16_t* __restrict__ k,
                                                          const bf16_t* __restrict__ v, bf16_t* __restrict__ o,
                                                          float* __restrict__ lse, int S, int H, int KV,
                                                          float scale_log2, int xcd, int64_t qis, int64_t kvs) {
  constexpr int BQ = 128;
  constexpr int TILE = 64 * 2 * D, STAGE = 2 * TILE;   // one 64-row K (or V) tile; K + V
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  int qb, hq, b;
  grid_decode(xcd, H, KV, qb, hq, b);  // longest causal rows first
  const int hk = hq / (H / KV);
  const int lane = threadIdx.x & 63, h = lane >> 5, l31 = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // provably wave-uniform
  const int q0 = qb * BQ;
  const int wq0 = q0 + 32 * w;  // first query of this wave
  // q / k / v token rows are qis / kvs elements apart (H*D / KV*D, or 3*H*D for the slices of
  // one packed qkv projection); o is written contiguous
  const int64_t qs = (int64_t)H * D, ks = kvs;
  const bf16_t* qp = q + (int64_t)b * S * qis + hq * D;
  const bf16_t* kp = k + (int64_t)b * S * ks + hk * D;
  const bf16_t* vp = v + (int64_t)b * S * ks + hk * D;

  const int qr = wq0 + l31;
  bf16x8 qf[D / 16];
#pragma unroll
  for (int s = 0; s < D / 16; ++s) qf[s] = load_frag(qp + (int64_t)min(qr, S - 1) * qis, s, h);
  const int kv_end = CAUSAL ? min(S, q0 + BQ) : S;
  const int ntiles = (kv_end + 63) / 64;
  f32x16 oacc[D / 32];
  float m = -1e30f, lsum = 0.f;
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt) oacc[dt] = f32x16{};

  const DmaPlan<64, 4, D> plan(ks, w, lane);
  const int64_t kv_bytes = ((int64_t)S * ks - hk * D) * 2;
  const rsrc_t krs = make_rsrc(kp, kv_bytes), vrs = make_rsrc(vp, kv_bytes);
  const uint32_t tile_bytes = (uint32_t)(64 * ks * 2);
  plan.issue(smem, krs, 0, w);
  plan.issue(smem + TILE, vrs, 0, w);
  wait_vm();
  __syncthreads();

  // Tiles below the workgroup's first query (and inside S) need no mask for
  // any wave: run them in a mask-free loop, the diagonal / tail tiles in a
  // second loop (two straight-line bodies allocate registers better than one
  // body with a masked and an unmasked branch).
  const int nfull = CAUSAL ? min(q0, S) / 64 : S / 64;
  // The loop body is unrolled over the two LDS stages so every LDS address is a
  // loop-invariant register plus an immediate (no per-read address VALU).
  auto run = [&](auto masked, int it0, int it1) {
    constexpr bool MASK = decltype(masked)::value;
    auto step = [&](int it, auto stage) {
      constexpr int ST = decltype(stage)::value;   // == it & 1
      const int kv0 = it * 64;
      if (it + 1 < ntiles) {  // stage 1-ST was released by the previous barrier
        plan.issue(smem + (1 - ST) * STAGE, krs, (it + 1) * tile_bytes, w);
        plan.issue(smem + (1 - ST) * STAGE + TILE, vrs, (it + 1) * tile_bytes, w);
      }
      const char* Ks = smem + ST * STAGE;
      if (!MASK || !CAUSAL || kv0 <= wq0 + 31)  // wave-uniform: tile visible to this wave
        fwd_tile<MASK, CAUSAL, D>(Ks, Ks + TILE, qf, oacc, m, lsum, kv0, qr, S, scale_log2, lane);
      wait_vm();
      __syncthreads();
    };
    int it = it0;
    if (it < it1 && (it & 1)) step(it++, std::integral_constant<int, 1>{});
#pragma unroll 1
    for (; it + 1 < it1; it += 2) {
      step(it, std::integral_constant<int, 0>{});
      step(it + 1, std::integral_constant<int, 1>{});
    }
    if (it < it1) step(it, std::integral_constant<int, 0>{});
  };
  run(std::integral_constant<bool, false>{}, 0, nfull);
  run(std::integral_constant<bool, true>{}, nfull, ntiles);
  const float ltot = xhalf_sum(lsum);
  if (qr < S) {
    store_accT(o + (int64_t)b * S * qs + (int64_t)qr * qs + hq * D, oacc, 1.f / ltot, h);
    if (h == 0) lse[((int64_t)b * H + hq) * S + qr] = (m + log2f(ltot)) * LN2;
  }
}

// ---------------------------------------------------------------------------
// forward, software-pipelined (cdna_hip_programming.md "4-wave, one-wave-per-
// SIMD" structure).  A workgroup = 4 waves = 256 queries of one head; a wave
// owns 64 queries as two 32-query column blocks (qb) that share every K and V
// fragment, so each LDS read feeds two MFMAs.  One wave per SIMD: the wave
// hides its own latency by running the softmax of one tile beside the matrix
// products of its neighbours.  Per 64-key tile j:
//   phase 1: S(j+1) = K(j+1) Q^T   (32 MFMAs) || exp / row-sum / bf16-pack of S(j), qb 1
//   phase 2: O^T += V(j)^T P(j)^T  (32 MFMAs) || row max of S(j+1), running-max update,
//                                                exp / row-sum / pack of S(j+1), qb 0
// so every MFMA gap carries <= ~5 VALU issues (cdna_hip_programming.md
// Appendix B 'Fused attention prefill'), and at most one S tile plus half of
// the next is live in fp32.  Register placement is pinned with asm MFMAs:
// S in VGPRs (softmax works in place), O and Q in AGPRs (only MFMAs touch them
// in the loop); each step is a sched_barrier region, so LDS reads are issued
// one (V) or two (K) steps ahead of their MFMAs.  K/V tiles stream through
// 4-slot LDS rings by LDS-DMA (K three tiles ahead, V two), one barrier per
// tile; the body is unrolled over the ring slots so every LDS address is a
// register plus an immediate.  Lazy rescale: the running max moves only when
// a row grew by > 2^8 (then O is rescaled after the tile's PV, l at once).
// ---------------------------------------------------------------------------
namespace fwd64 {
constexpr int NS = 4;         // ring slots
constexpr int TB = 16384;     // one 64-row x 256-B tile

// hipcc pads nothing inside asm: MFMA D -> VALU read needs 18 wait states
// (fence_d), a VALU / v_accvgpr_write result -> MFMA operand 2 (fence_op);
// chained MFMAs that take their own D whole as C need none.
__device__ __forceinline__ void mfma_s0(f32x16& d, const bf16x8& kf, const bf16x8& qf) {
  asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(d) : "v"(kf), "a"(qf));
}
__device__ __forceinline__ void mfma_s(f32x16& d, const bf16x8& kf, const bf16x8& qf) {
  asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(d) : "v"(kf), "a"(qf));
}
__device__ __forceinline__ void mfma_o(f32x16& acc, const bf16x8& vf, const bf16x8& pb) {
  asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(vf), "v"(pb));
}
__device__ __forceinline__ void fence_d(f32x16 (&x)[2][2]) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 4" : "+v"(x[0][0]), "+v"(x[0][1]), "+v"(x[1][0]), "+v"(x[1][1]));
}
__device__ __forceinline__ void fence_d_acc(f32x16 (&o)[4]) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 4" : "+a"(o[0]), "+a"(o[1]), "+a"(o[2]), "+a"(o[3]));
}
__device__ __forceinline__ void fence_acc(f32x16 (&o)[4]) {
  asm volatile("s_nop 1" : "+a"(o[0]), "+a"(o[1]), "+a"(o[2]), "+a"(o[3]));
}
__device__ __forceinline__ void fence_op(bf16x8 (&p)[2][2][2]) {
  asm volatile("s_nop 1" : "+v"(p[0][0][0]), "+v"(p[0][0][1]), "+v"(p[0][1][0]), "+v"(p[0][1][1]),
               "+v"(p[1][0][0]), "+v"(p[1][0][1]), "+v"(p[1][1][0]), "+v"(p[1][1][1]));
}
// v_max3 beside MFMA results (asm: hipcc otherwise inserts canonicalising v_max
// before fmaxf on them).  Its inputs are MFMA results behind fence_d and
// plain VALU (mask) values -- never a transcendental result: a trans -> VALU
// read needs a wait state that hipcc does not pad for an asm consumer (an asm
// v_add after v_exp read the pre-exp value).  Row sums are plain adds, one
// query block per soft() call, pinned after it (no adjacent independent chains
// for hipcc to SLP-pack into v_pk_add_f32, ~+22 cycles each beside MFMAs).
__device__ __forceinline__ float max3(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

struct State {
  bf16x8 qf[2][8];            // Q fragments of the two 32-query blocks (AGPRs)
  f32x16 o[2][4];             // O^T accumulators (d = 32*dt + row, query = lane & 31; AGPRs)
  f32x16 s[2][2][2];          // S tiles by tile parity: [buf][qb][key half t]
  bf16x8 pb[2][2][2][2];      // P tiles as bf16 B operands: [buf][qb][t][s2]
  bf16x8 kf[3];               // K fragment ring (read two steps ahead)
  bf16x8 vf[2];               // V fragment ring (read one step ahead)
  float m[2], ls[2], al[2];   // running max (scaled log2), row sums, pending O rescale
};

#define EDL_SB() __builtin_amdgcn_sched_barrier(0)

// LDS addressing: V ring at [0, 64K), K ring at [64K, 128K).  Every read is a
// per-lane base register plus a compile-time immediate (slot, key half, s2)
// that stays below the 16-bit ds offset limit: K bases hold 64K + the lane's
// swizzled row/chunk for each k-step s (8 registers), V bases the lane's
// transposed-read piece for each (dt, lo/hi) (8 registers).
struct Lds {
  uint32_t k[8];
  uint32_t v[4][2];
};

__device__ __forceinline__ Lds lds_bases(const char* smem, int lane) {
  Lds a;
  const uint32_t base = (uint32_t)(uintptr_t)(const lds_char*)smem;
  const int h = lane >> 5, l31 = lane & 31;
#pragma unroll
  for (int s = 0; s < 8; ++s) a.k[s] = base + NS * TB + swz(l31, 2 * s + h);
  const int i = lane & 15, qq = i >> 2, p = i & 3;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    const int col = dt * 32 + ((lane >> 4) & 1) * 16 + 4 * p;
    const int c = col >> 3, half = (col >> 2) & 1;
    a.v[dt][0] = base + swz(4 * h + qq, c) + half * 8;
    a.v[dt][1] = base + swz(4 * h + 8 + qq, c) + half * 8;
  }
#pragma unroll
  for (int s = 0; s < 8; ++s) asm volatile("" : "+v"(a.k[s]));   // keep them plain registers
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) asm volatile("" : "+v"(a.v[dt][0]), "+v"(a.v[dt][1]));
  return a;
}

// K fragment of step k (key half k>>3, k-step k&7) of ring slot `slot`
__device__ __forceinline__ void kread(State& st, const Lds& a, int slot, int k) {
  st.kf[k % 3] = *(const lds_bf16x8*)(uintptr_t)(a.k[k & 7] + slot * TB + (k >> 3) * 8192);
}
// V^T fragment of PV step k (key half k>>3, s2 = (k>>2)&1, dt = k&3) of ring slot `slot`
__device__ __forceinline__ void vread(State& st, const Lds& a, int slot, int k) {
  const uint32_t off = slot * TB + (32 * (k >> 3) + 16 * ((k >> 2) & 1)) * 256;
  const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(uintptr_t)(a.v[k & 3][0] + off));
  const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(uintptr_t)(a.v[k & 3][1] + off));
  st.vf[k & 1] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

// exp / row sum of scores f (0..31, = 16 t + i) of query block qb of S(buf); packs
// every completed group of 8 into pb[buf][qb]
__device__ __forceinline__ void soft(State& st, int buf, int qb, int f0, int f1, float sl2, float negm) {
#pragma unroll
  for (int f = f0; f < f1; ++f) {
    const int t = f >> 4, i = f & 15;
    const float p = fast_exp2(__builtin_fmaf(st.s[buf][qb][t][i], sl2, negm));
    st.s[buf][qb][t][i] = p;
    st.ls[qb] += p;
    if ((f & 7) == 7) st.pb[buf][qb][t][(f >> 3) & 1] = acc_to_b(st.s[buf][qb][t], (f >> 3) & 1);
  }
  // pin the sum here: otherwise hipcc sinks the add chain to the loop latch and keeps
  // every p alive (spilled) until then
  asm volatile("" : "+v"(st.ls[qb]));
}

// phase 1: S(nb) = K Q^T (K fragments 0, 1 already read) || softmax of S(cb), qb 1
__device__ __forceinline__ void phase1(State& st, int nb, int cb, const Lds& a, int kslot, float sl2,
                                       bool soft1) {
  const float negm = -st.m[1];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    if (k + 2 < 16) kread(st, a, kslot, k + 2);
    const int t = k >> 3, s = k & 7;
    if (s == 0) {
      mfma_s0(st.s[nb][0][t], st.kf[k % 3], st.qf[0][s]);
      mfma_s0(st.s[nb][1][t], st.kf[k % 3], st.qf[1][s]);
    } else {
      mfma_s(st.s[nb][0][t], st.kf[k % 3], st.qf[0][s]);
      mfma_s(st.s[nb][1][t], st.kf[k % 3], st.qf[1][s]);
    }
    if (soft1) soft(st, cb, 1, 2 * k, 2 * k + 2, sl2, negm);
    EDL_SB();
  }
}

// phase 2: O += V^T P(cb)^T (V fragment 0 already read) || max of S(nb) (steps 0-3),
// running-max update, softmax of S(nb), qb 0 (steps 4-15).  S(nb) is fenced.
__device__ __forceinline__ void phase2(State& st, int nb, int cb, const Lds& a, int vslot, float sl2, bool next) {
  float mx[2][2];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    if (k + 1 < 16) vread(st, a, vslot, k + 1);
    const int t = k >> 3, s2 = (k >> 2) & 1, dt = k & 3;
    mfma_o(st.o[0][dt], st.vf[k & 1], st.pb[cb][0][t][s2]);
    mfma_o(st.o[1][dt], st.vf[k & 1], st.pb[cb][1][t][s2]);
    if (next) {
      if (k < 4) {   // 4 registers per (qb, t) per step
#pragma unroll
        for (int qb = 0; qb < 2; ++qb)
#pragma unroll
          for (int tt = 0; tt < 2; ++tt) {
            const f32x16& x = st.s[nb][qb][tt];
            mx[qb][tt] = k == 0 ? max3(max3(x[0], x[1], x[2]), x[3], x[3])
                                : max3(max3(mx[qb][tt], x[4 * k], x[4 * k + 1]), x[4 * k + 2], x[4 * k + 3]);
          }
      }
      if (k == 3) {  // running-max update (per row; l at once, O after this tile's PV)
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) {
          const float mxs = xhalf_max(fmaxf(mx[qb][0], mx[qb][1])) * sl2;
          const float mnew = mxs > st.m[qb] + 8.f ? fmaxf(st.m[qb], mxs) : st.m[qb];
          const float alpha = fast_exp2(st.m[qb] - mnew);
          st.m[qb] = mnew;
          st.ls[qb] *= alpha;
          st.al[qb] *= alpha;
        }
      }
      if (k >= 4) soft(st, nb, 0, (32 * (k - 4)) / 12, (32 * (k - 3)) / 12, sl2, -st.m[0]);
    }
    EDL_SB();
  }
}

// pending O rescale (rare: only when some row's max moved)
__device__ __forceinline__ void apply_rescale(State& st) {
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    if (__any(st.al[qb] != 1.f)) {
      fence_d_acc(st.o[qb]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) st.o[qb][dt] *= st.al[qb];
      fence_acc(st.o[qb]);
    }
    st.al[qb] = 1.f;
  }
}

// scores of keys past min(query, S-1) -> -inf (diagonal / tail tiles only)
template <bool CAUSAL>
__device__ __forceinline__ void mask(State& st, int buf, int kv0, int wq0, int S, int h) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const int lim = CAUSAL ? min(wq0 + 32 * qb + (lane & 31), S - 1) : S - 1;
    const int rel = lim - kv0 - 4 * h;   // key - kv0 - 4h = 32t + (i&3) + 8(i>>2)
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i)
        if (32 * t + (i & 3) + 8 * (i >> 2) > rel) st.s[buf][qb][t][i] = -INFINITY;
  }
}

// s_waitcnt vmcnt(N) for the LDS-DMA pieces still allowed in flight
__device__ __forceinline__ void wait_vm_n(int n) {
  if (n >= 8)
    __builtin_amdgcn_s_waitcnt(0x0F78);
  else if (n >= 4)
    __builtin_amdgcn_s_waitcnt(0x0F74);
  else
    __builtin_amdgcn_s_waitcnt(0x0F70);
}
}  // namespace fwd64

template <bool CAUSAL>
__global__ __launch_bounds__(256, 1) void attn_fwd64_kernel(const bf16_t* __restrict__ q, const bf16_t* __restrict__ k,
                                                            const bf16_t* __restrict__ v, bf16_t* __restrict__ o,
                                                            float* __restrict__ lse, int S, int H, int KV,
                                                            float sl2, int64_t qis, int64_t kvs) {
  using namespace fwd64;
  constexpr int BQ = 256;
  __shared__ __attribute__((aligned(16))) char smem[2 * NS * TB];   // K ring, then V ring (one array)
  const int qblk = gridDim.x - 1 - blockIdx.x;  // longest causal rows first
  const int hq = blockIdx.y, b = blockIdx.z, hk = hq / (H / KV);
  const int lane = threadIdx.x & 63, h = lane >> 5, l31 = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int q0 = qblk * BQ, wq0 = q0 + 64 * w;
  const int64_t qs = (int64_t)H * HD, ks = kvs;   // input row strides as in attn_fwd_kernel
  const bf16_t* qp = q + (int64_t)b * S * qis + hq * HD;
  const bf16_t* kp = k + (int64_t)b * S * ks + hk * HD;
  const bf16_t* vp = v + (int64_t)b * S * ks + hk * HD;

  State st;
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const bf16_t* rowp = qp + (int64_t)min(wq0 + 32 * qb + l31, S - 1) * qis;
#pragma unroll
    for (int s = 0; s < 8; ++s) st.qf[qb][s] = load_frag(rowp, s, h);
    st.m[qb] = -1e30f;
    st.ls[qb] = 0.f;
    st.al[qb] = 1.f;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) st.o[qb][dt] = f32x16{};
  }
  const int kv_end = CAUSAL ? min(S, q0 + BQ) : S;
  const int nt = (kv_end + 63) / 64;
  const int nfull = CAUSAL ? min(q0, S) / 64 : S / 64;   // tiles that need no mask for any wave

  const DmaPlan<64, 4> plan(ks, w, lane);
  const int64_t kv_bytes = ((int64_t)S * ks - hk * HD) * 2;
  const rsrc_t krs = make_rsrc(kp, kv_bytes), vrs = make_rsrc(vp, kv_bytes);
  const uint32_t tile_bytes = (uint32_t)(64 * ks * 2);
  char* const Vr = smem;             // V ring [0, 64K)
  char* const Kr = smem + NS * TB;   // K ring [64K, 128K)
  // K(i) -> K slot i%4, three tiles ahead; V(i) -> V slot i%4, two tiles ahead
  plan.issue(Kr, krs, 0, w);
  if (nt > 1) plan.issue(Kr + TB, krs, tile_bytes, w);
  if (nt > 2) plan.issue(Kr + 2 * TB, krs, 2 * tile_bytes, w);
  plan.issue(Vr, vrs, 0, w);
  if (nt > 1) plan.issue(Vr + TB, vrs, tile_bytes, w);
  wait_vm();
  __syncthreads();
  // Q fragments and the zeroed O -> AGPRs (v_accvgpr_write -> MFMA operand: 2 wait states)
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
#pragma unroll
    for (int s = 0; s < 8; s += 4)
      asm volatile("s_nop 1" : "+a"(st.qf[qb][s]), "+a"(st.qf[qb][s + 1]), "+a"(st.qf[qb][s + 2]),
                   "+a"(st.qf[qb][s + 3]));
    fence_acc(st.o[qb]);
  }

  const Lds la = lds_bases(smem, lane);
  // prologue: S(0), its row max, the running max, softmax of S(0) qb 0
  kread(st, la, 0, 0);
  kread(st, la, 0, 1);
  phase1(st, 0, 1, la, 0, sl2, false);
  fence_d(st.s[0]);
  if (0 >= nfull) mask<CAUSAL>(st, 0, 0, wq0, S, h);
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    float a = st.s[0][qb][0][0];
#pragma unroll
    for (int f = 1; f < 32; ++f) a = fmaxf(a, st.s[0][qb][f >> 4][f & 15]);
    st.m[qb] = xhalf_max(a) * sl2;   // O = 0, l = 0: nothing to rescale
  }
  soft(st, 0, 0, 0, 32, sl2, -st.m[0]);

  // iteration j (ring slot ST = j % 4, tile parity B = j % 2): K(j+1), V(j) resident
  auto iter = [&](int j, auto stage) {
    constexpr int ST = decltype(stage)::value;
    constexpr int B = ST & 1;
    int issued = 0;
    kread(st, la, (ST + 1) % NS, 0);
    kread(st, la, (ST + 1) % NS, 1);
    if (j + 3 < nt) {
      plan.issue(Kr + ((ST + 3) % NS) * TB, krs, (uint32_t)(j + 3) * tile_bytes, w);
      issued += 4;
    }
    EDL_SB();
    phase1(st, B ^ 1, B, la, (ST + 1) % NS, sl2, true);
    if (j + 2 < nt) {
      plan.issue(Vr + ((ST + 2) % NS) * TB, vrs, (uint32_t)(j + 2) * tile_bytes, w);
      issued += 4;
    }
    vread(st, la, ST, 0);
    fence_op(st.pb[B]);
    fence_d(st.s[B ^ 1]);
    EDL_SB();
#ifndef EDL_ISA_HOTPATH  // (ISA audits of the steady-state body compile the rare paths out)
    if (j + 1 >= nfull) mask<CAUSAL>(st, B ^ 1, (j + 1) * 64, wq0, S, h);
#endif
    phase2(st, B ^ 1, B, la, ST, sl2, true);
#ifndef EDL_ISA_HOTPATH
    apply_rescale(st);
#endif
    wait_vm_n(issued);
    __builtin_amdgcn_s_barrier();
  };
  int j = 0;
#pragma unroll 1
  for (; j + 4 <= nt - 1; j += 4) {
    iter(j, std::integral_constant<int, 0>{});
    iter(j + 1, std::integral_constant<int, 1>{});
    iter(j + 2, std::integral_constant<int, 2>{});
    iter(j + 3, std::integral_constant<int, 3>{});
  }
  if (j < nt - 1) iter(j++, std::integral_constant<int, 0>{});
  if (j < nt - 1) iter(j++, std::integral_constant<int, 1>{});
  if (j < nt - 1) iter(j++, std::integral_constant<int, 2>{});
  // drain: softmax of the last tile's qb 1, its PV (runtime slot; once per workgroup),
  // epilogue.  Each parity branch ends with its own fence + stores so that no O value
  // is live across the join: hipcc would otherwise insert v_accvgpr_mov phi copies
  // right behind the last (asm, opaque) MFMA and read its result before it lands.
  {
    const int vslot = (nt - 1) % NS;
    auto fin = [&](auto bufc) {
      constexpr int CB = decltype(bufc)::value;
      soft(st, CB, 1, 0, 32, sl2, -st.m[1]);
      fence_op(st.pb[CB]);
      vread(st, la, vslot, 0);
      phase2(st, CB ^ 1, CB, la, vslot, sl2, false);
      fence_d_acc(st.o[0]);
      fence_d_acc(st.o[1]);
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        const int qr = wq0 + 32 * qb + l31;
        const float ltot = xhalf_sum(st.ls[qb]);
        if (qr < S) {
          store_accT(o + (int64_t)b * S * qs + (int64_t)qr * qs + hq * HD, st.o[qb], 1.f / ltot, h);
          if (h == 0) lse[((int64_t)b * H + hq) * S + qr] = (st.m[qb] + log2f(ltot)) * LN2;
        }
      }
    };
    if ((nt - 1) & 1)
      fin(std::integral_constant<int, 1>{});
    else
      fin(std::integral_constant<int, 0>{});
  }
}

// ---------------------------------------------------------------------------
// backward preprocess: delta = rowsum(dO * O)   (D/8 lanes per row, 16 B each)
// ---------------------------------------------------------------------------
template <int D>
__global__ __launch_bounds__(256) void attn_bwd_delta_kernel(const bf16_t* __restrict__ o,
                                                             const bf16_t* __restrict__ dout,
                                                             const float* __restrict__ lse,
                                                             float* __restrict__ delta, int S, int H,
                                                             int64_t nrows) {
  constexpr int LPR = D / 8;
  const int64_t row = ((int64_t)blockIdx.x * 256 + threadIdx.x) / LPR;  // row = (b*S + s)*H + h
  const int c = threadIdx.x % LPR;
  float acc = 0.f;
  if (row < nrows) {
    float a[8], d[8];
    unpack8(reinterpret_cast<const u32x4*>(o + row * D)[c], a);
    unpack8(reinterpret_cast<const u32x4*>(dout + row * D)[c], d);
#pragma unroll
    for (int i = 0; i < 8; ++i) acc += a[i] * d[i];
  }
#pragma unroll
  for (int off = LPR / 2; off > 0; off >>= 1) acc += __shfl_xor(acc, off, LPR);
  if (c == 0 && row < nrows) {
    const int64_t hh = row % H, tok = row / H, s = tok % S, b = tok / S;
    const int64_t i = (b * H + hh) * S + s;
    delta[i] = acc;
    delta[nrows + i] = -lse[i] * LOG2E;  // row constant of the exp2 in both bwd kernels
  }
}

// ---------------------------------------------------------------------------
// backward: dK, dV.  A workgroup owns 128 keys of one KV head (a wave 32 keys,
// K/V in registers, dK^T/dV^T accumulators resident) and sweeps 64-query
// tiles (two 32-row sub-slices) of every query head of the GQA group.
// LDS per stage: Q tile, dO tile, -lse*log2(e) and delta for the 64 rows.
// ---------------------------------------------------------------------------
// Issue order S, dP (16 back-to-back MFMAs), then exp(S) under the dP MFMAs,
// dV += dO^T P under which dS = P (dP - delta) runs, then dK += Q^T dS.
template <bool MASK, bool CAUSAL, int D>
__device__ __forceinline__ void dkdv_slice(const char* Qs, const char* Ds, const float* NL, const float* DL, int rb,
                                           const bf16x8 (&kf)[D / 16], const bf16x8 (&vf)[D / 16],
                                           f32x16 (&dka)[D / 32], f32x16 (&dva)[D / 32], int qs0, int mykey, int S,
                                           float sl2, int lane) {
  const int h = lane >> 5, l31 = lane & 31;
  f32x16 sa = f32x16{}, dp = f32x16{};
#pragma unroll
  for (int s = 0; s < D / 16; ++s) sa = mfma(row_read<D>(Qs, rb + l31, s, h), kf[s], sa);
#pragma unroll
  for (int s = 0; s < D / 16; ++s) dp = mfma(row_read<D>(Ds, rb + l31, s, h), vf[s], dp);
  // accumulator register i <-> query row rb + acc_row(i, h): rows 8g+4h .. +3 are contiguous
  f32x4 nl[4], dl[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    nl[g] = *reinterpret_cast<const f32x4*>(NL + rb + 8 * g + 4 * h);
    dl[g] = *reinterpret_cast<const f32x4*>(DL + rb + 8 * g + 4 * h);
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    float p = fast_exp2(__builtin_fmaf(sa[i], sl2, nl[i >> 2][i & 3]));
    if (MASK) {
      const int qi = qs0 + acc_row(i, h);
      if (qi >= S || mykey >= S || (CAUSAL && mykey > qi)) p = 0.f;
    }
    sa[i] = p;
  }
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    const bf16x8 pb = acc_to_b(sa, s2);
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt) dva[dt] = mfma(tr_read<D>(Ds, rb + 16 * s2 + 4 * h, dt, lane), pb, dva[dt]);
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) dp[i] = sa[i] * (dp[i] - dl[i >> 2][i & 3]);
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    const bf16x8 db = acc_to_b(dp, s2);
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt) dka[dt] = mfma(tr_read<D>(Qs, rb + 16 * s2 + 4 * h, dt, lane), db, dka[dt]);
  }
}

// OCC = waves per SIMD the register budget is cut for: 1 keeps every K/V
// fragment resident (no spill); 2 doubles the latency hiding but reloads six
// fragments per slice from scratch.  Chosen at launch (EDL_ATTN_DKDV_OCC).
template <bool CAUSAL, int OCC, int D = 128>
__global__ __launch_bounds__(256, OCC) void attn_bwd_dkdv_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    const bf16_t* __restrict__ dout, const float* __restrict__ lse, const float* __restrict__ delta,
    bf16_t* __restrict__ dk, bf16_t* __restrict__ dv, int S, int H, int KV, float scale_log2, float scale,
    int64_t dkvs, int64_t kvs) {
  constexpr int QT = 64;  // queries per staged tile
  constexpr int TILE = QT * 2 * D, STAGE = 2 * TILE;
  // 2 stages x (Q tile + dO tile) + 2 x (-lse2, delta) x 64 floats
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE + 2 * 512];
  const int kb = blockIdx.x, hk = blockIdx.y, b = blockIdx.z;
  const int lane = threadIdx.x & 63, h = lane >> 5, l31 = lane & 31;
  const int w = threadIdx.x >> 6;
  const int group = H / KV;
  const int64_t qs = (int64_t)H * D, ks = kvs;   // q / dO rows contiguous; k / v rows kvs apart
  const int mykey = kb * 128 + 32 * w + l31;
  const int64_t krow_off = (int64_t)b * S * ks + (int64_t)min(mykey, S - 1) * ks + hk * D;
  bf16x8 kf[D / 16], vf[D / 16];
#pragma unroll
  for (int s = 0; s < D / 16; ++s) {
    kf[s] = load_frag(k + krow_off, s, h);
    vf[s] = load_frag(v + krow_off, s, h);
  }
  f32x16 dka[D / 32], dva[D / 32];
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt) {
    dka[dt] = f32x16{};
    dva[dt] = f32x16{};
  }
  const int nqt = (S + QT - 1) / QT;
  const int qt0 = CAUSAL ? (kb * 128) / QT : 0;
  const int per_head = nqt - qt0;
  const int total = per_head * group;
  const int wave_key_lo = kb * 128 + 32 * w;

  const int64_t nBHS = (int64_t)gridDim.z * H * S;  // delta = [delta | -lse*log2e]
  const DmaPlan<QT, 4, D> plan(qs, w, lane);
  auto fetch = [&](int j, int st) {
    const int hq = hk * group + j / per_head;
    const int q0 = (qt0 + j % per_head) * QT;
    char* base = smem + st * STAGE;
    const int64_t off = (int64_t)b * S * qs + hq * D, nbytes = ((int64_t)S * qs - hq * D) * 2;
    const uint32_t soff = (uint32_t)(q0 * qs * 2);
    plan.issue(base, make_rsrc(q + off, nbytes), soff, w);
    plan.issue(base + TILE, make_rsrc(dout + off, nbytes), soff, w);
    float* lf = reinterpret_cast<float*>(smem + 2 * STAGE + st * 512);
    const int64_t row0 = ((int64_t)b * H + hq) * S;
    if (w == 0) dma_f32x64(lf, make_rsrc(delta + nBHS + row0, (int64_t)S * 4), q0, lane);
    if (w == 1) dma_f32x64(lf + QT, make_rsrc(delta + row0, (int64_t)S * 4), q0, lane);
  };
  if (total > 0) fetch(0, 0);
  wait_vm();
  __syncthreads();
#pragma unroll 1
  for (int j = 0; j < total; ++j) {
    if (j + 1 < total) fetch(j + 1, (j + 1) & 1);
    const int st = j & 1;
    const char* Qs = smem + st * STAGE;
    const char* Ds = Qs + TILE;
    const float* NL = reinterpret_cast<const float*>(smem + 2 * STAGE + st * 512);
    const int q0 = (qt0 + j % per_head) * QT;
#pragma unroll
    for (int sub = 0; sub < QT / 32; ++sub) {
      const int qs0 = q0 + 32 * sub;
      if (CAUSAL && qs0 + 31 < wave_key_lo) continue;  // wave-uniform: all masked
      const bool mask = (qs0 + 32 > S) || (wave_key_lo + 32 > S) || (CAUSAL && wave_key_lo + 31 > qs0);
      if (mask)
        dkdv_slice<true, CAUSAL, D>(Qs, Ds, NL, NL + QT, 32 * sub, kf, vf, dka, dva, qs0, mykey, S, scale_log2,
                                    lane);
      else
        dkdv_slice<false, CAUSAL, D>(Qs, Ds, NL, NL + QT, 32 * sub, kf, vf, dka, dva, qs0, mykey, S, scale_log2,
                                     lane);
    }
    wait_vm();
    __syncthreads();
  }
  if (mykey < S) {
    store_accT(dk + ((int64_t)b * S + mykey) * dkvs + hk * D, dka, scale, h);
    store_accT(dv + ((int64_t)b * S + mykey) * dkvs + hk * D, dva, 1.f, h);
  }
}

// ---------------------------------------------------------------------------
// backward: dK, dV with 64 keys per wave.  The 32-key kernel above is LDS-
// bandwidth-bound: every 32x32x16 MFMA consumes one 1-KiB LDS fragment, which
// is exactly the CU's LDS rate at full MFMA rate (prefetching the fragments
// earlier measured 4.5 % SLOWER, profiles/r01_attn_dkdv_ab.txt).  Here a wave
// owns two 32-key blocks, so every Q / dO fragment read from LDS feeds two
// MFMAs.  Registers: K fragments 64 VGPRs, dK/dV accumulators 256 (AGPRs),
// S/dP 64; V is read from LDS -> one wave per SIMD, as before.  A
// workgroup (4 waves) owns 256 keys of one KV head.  Measured at the 8k causal
// Llama shape: 1.35 ms (incl. the partial-sum reduce) vs 2.25 ms for the
// 32-key kernel (profiles/r01_attn_dkdv_ab.txt); EDL_ATTN_DKDV=32 selects it.
// ---------------------------------------------------------------------------
// S / dP MFMAs of the dK/dV-64 kernel with their results pinned to VGPRs.  With the
// builtin, the compiler puts every MFMA result in AGPRs, and S/dP (64) plus the dK/dV
// accumulators (256) do not fit the 256 AGPRs: it shuffled 64 accumulators through
// ~200 v_accvgpr moves per slice.  hipcc pads nothing inside asm: the first MFMA of a
// chain takes C = 0 (no VALU-written C), chained MFMAs read C = their own D (0 wait
// states), and mfma_d_fence pads the MFMA D -> VALU read once after both chains.
__device__ __forceinline__ void mfma_v_first(f32x16& d, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(d) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mfma_v(f32x16& d, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(d) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mfma_d_fence(f32x16 (&x)[2], f32x16 (&y)[2]) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 4" : "+v"(x[0]), "+v"(x[1]), "+v"(y[0]), "+v"(y[1]));
}

// Software-pipelined form of the slice below (EDL_ATTN_DKDV=64p).  The plain form reads each
// fragment right before its MFMAs, and the compiler puts an lgkmcnt(0) in front of every MFMA
// pair: the LDS latency is exposed 40+ times per slice (the ISA of the unmasked loop: 45
// s_waitcnt for 64 MFMAs; the kernel ran at 36 % of the MFMA peak, 0.9 PF/s).  Here
//  * S = Q K^T and dP = dO V^T run in ONE k-loop: 4 fragment reads + 4 MFMAs per k-step, the
//    next k-step's 4 reads issued before this step's MFMAs (128 MFMA cycles cover them);
//  * dV += dO^T P and dK += Q^T dS read their transposed fragments one MFMA pair ahead;
// each step is a sched_barrier region, so the reads stay ahead of the MFMAs they feed.
__device__ __forceinline__ void mfma_d_fence2(f32x16 (&x)[2]) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 4" : "+v"(x[0]), "+v"(x[1]));
}

template <bool MASK, bool CAUSAL, int D>
__device__ __forceinline__ void dkdv64p_slice(const char* Qs, const char* Ds, const float* NL,
                                              const float* DL, int rb, const bf16x8 (&kf)[2][D / 16],
                                              const char* Vw, f32x16 (&dka)[2][D / 32], f32x16 (&dva)[2][D / 32],
                                              int qs0, int key0, int S,
                                              float sl2, int lane) {
  const int h = lane >> 5, l31 = lane & 31;
  f32x16 sa[2], dp[2];
  uint32_t vo = (uint32_t)(uintptr_t)(lds_char*)Vw;
  asm volatile("" : "+v"(vo));
  const lds_char* Vl = (const lds_char*)(uintptr_t)vo;
  constexpr int NS = D / 16, NDT = D / 32;
#define EDL_SB() __builtin_amdgcn_sched_barrier(0)
  // Softmax terms and dS per quarter (one key tile t, one row group g = accumulator registers
  // 4g .. 4g+3; groups 0-1 feed the bf16 operands of k-half s2 = 0, groups 2-3 those of s2 = 1)
  auto expq = [&](int g, int t, const f32x4& nl) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float x = fast_exp2(__builtin_fmaf(sa[t][4 * g + e], sl2, nl[e]));
      if (MASK) {
        const int mykey = key0 + 32 * t + l31, qi = qs0 + acc_row(4 * g + e, h);
        if (qi >= S || mykey >= S || (CAUSAL && mykey > qi)) x = 0.f;
      }
      sa[t][4 * g + e] = x;
    }
  };
  auto dsq = [&](int g, int t, const f32x4& dl) {
#pragma unroll
    for (int e = 0; e < 4; ++e) dp[t][4 * g + e] = sa[t][4 * g + e] * (dp[t][4 * g + e] - dl[e]);
  };
  auto ld4 = [&](const float* base, int g) { return *reinterpret_cast<const f32x4*>(base + rb + 8 * g + 4 * h); };
  auto trq = [&](const char* T, int i) { return tr_read<D>(T, rb + 16 * (i / NDT) + 4 * h, i % NDT, lane); };

  // phase 1a: S = Q K^T, the next k-step's Q fragment read ahead of this step's MFMAs
  bf16x8 fq[2];
  fq[0] = row_read<D>(Qs, rb + l31, 0, h);
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    if (s + 1 < NS) fq[(s + 1) & 1] = row_read<D>(Qs, rb + l31, s + 1, h);
    EDL_SB();
    if (s == 0) {
      mfma_v_first(sa[0], fq[0], kf[0][0]);
      mfma_v_first(sa[1], fq[0], kf[1][0]);
    } else {
      mfma_v(sa[0], fq[s & 1], kf[0][s]);
      mfma_v(sa[1], fq[s & 1], kf[1][s]);
    }
    EDL_SB();
  }
  // phase 1b: dP = dO V^T (reads one k-step ahead)  ||  P = exp2(S sl2 - lse log2e), a quarter
  // per MFMA: S is final here, so the softmax runs under the dP MFMAs instead of after them
  bf16x8 fd[2], fv0[2], fv1[2];
  auto rdp = [&](int s, int b) {
    fd[b] = row_read<D>(Ds, rb + l31, s, h);
    fv0[b] = *(lds_bf16x8*)(Vl + swzd<D>(l31, 2 * s + h));
    fv1[b] = *(lds_bf16x8*)(Vl + swzd<D>(32 + l31, 2 * s + h));
  };
  rdp(0, 0);
  f32x4 nl[4] = {ld4(NL, 0), ld4(NL, 1), ld4(NL, 2), ld4(NL, 3)};
  mfma_d_fence2(sa);
  EDL_SB();
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int b = s & 1;
    if (s + 1 < NS) rdp(s + 1, b ^ 1);
    EDL_SB();
    if (s == 0) mfma_v_first(dp[0], fd[0], fv0[0]); else mfma_v(dp[0], fd[b], fv0[b]);
    EDL_SB();
    expq(s >> 1, s & 1, nl[s >> 1]);
    EDL_SB();
    if (s == 0) mfma_v_first(dp[1], fd[0], fv1[0]); else mfma_v(dp[1], fd[b], fv1[b]);
    EDL_SB();
  }
  const bf16x8 p0[2] = {acc_to_b(sa[0], 0), acc_to_b(sa[1], 0)};
  const bf16x8 p1[2] = {acc_to_b(sa[0], 1), acc_to_b(sa[1], 1)};
  bf16x8 ta[2];
  ta[0] = trq(Ds, 0);
  f32x4 dq[2] = {ld4(DL, 0), ld4(DL, 1)};
  mfma_d_fence2(dp);
  EDL_SB();
  // phase 2: dV += dO^T P (k-half 0)  ||  dS = P (dP - delta), groups 0-1
#pragma unroll
  for (int i = 0; i < NDT; ++i) {
    ta[(i + 1) & 1] = trq(Ds, i + 1);
    EDL_SB();
    dva[0][i] = mfma(ta[i & 1], p0[0], dva[0][i]);
    EDL_SB();
    dsq(i >> 1, i & 1, dq[i >> 1]);
    EDL_SB();
    dva[1][i] = mfma(ta[i & 1], p0[1], dva[1][i]);
    EDL_SB();
  }
  const bf16x8 d0[2] = {acc_to_b(dp[0], 0), acc_to_b(dp[1], 0)};
  dq[0] = ld4(DL, 2);
  dq[1] = ld4(DL, 3);
  EDL_SB();
  // dV k-half 1  ||  dS groups 2-3
#pragma unroll
  for (int i = NDT; i < 2 * NDT; ++i) {
    ta[(i + 1) & 1] = i + 1 < 2 * NDT ? trq(Ds, i + 1) : trq(Qs, 0);
    EDL_SB();
    dva[0][i - NDT] = mfma(ta[i & 1], p1[0], dva[0][i - NDT]);
    EDL_SB();
    dsq(2 + ((i - NDT) >> 1), i & 1, dq[(i - NDT) >> 1]);
    EDL_SB();
    dva[1][i - NDT] = mfma(ta[i & 1], p1[1], dva[1][i - NDT]);
    EDL_SB();
  }
  const bf16x8 d1[2] = {acc_to_b(dp[0], 1), acc_to_b(dp[1], 1)};
  EDL_SB();
  // phase 3: dK += Q^T dS
#pragma unroll
  for (int i = 0; i < 2 * NDT; ++i) {
    if (i + 1 < 2 * NDT) ta[(i + 1) & 1] = trq(Qs, i + 1);
    EDL_SB();
    const bf16x8* dsv = i < NDT ? d0 : d1;
    dka[0][i % NDT] = mfma(ta[i & 1], dsv[0], dka[0][i % NDT]);
    dka[1][i % NDT] = mfma(ta[i & 1], dsv[1], dka[1][i % NDT]);
    EDL_SB();
  }
#undef EDL_SB
#define EDL_SB() __builtin_amdgcn_sched_barrier(0)
}

template <bool MASK, bool CAUSAL, int D>
__device__ __forceinline__ void dkdv64_slice(const char* Qs, const char* Ds, const float* NL,
                                             const float* DL, int rb, const bf16x8 (&kf)[2][D / 16],
                                             const char* Vw, f32x16 (&dka)[2][D / 32], f32x16 (&dva)[2][D / 32],
                                             int qs0, int key0, int S,
                                             float sl2, int lane) {
  const int h = lane >> 5, l31 = lane & 31;
  f32x16 sa[2], dp[2];
  // V is read from LDS in every slice: the opaque offset stops the compiler from hoisting
  // the loop-invariant reads into (64 more) registers
  uint32_t vo = (uint32_t)(uintptr_t)(lds_char*)Vw;
  asm volatile("" : "+v"(vo));
  const lds_char* Vl = (const lds_char*)(uintptr_t)vo;
#pragma unroll
  for (int s = 0; s < D / 16; ++s) {
    const bf16x8 a = row_read<D>(Qs, rb + l31, s, h);
    if (s == 0) {
      mfma_v_first(sa[0], a, kf[0][s]);
      mfma_v_first(sa[1], a, kf[1][s]);
    } else {
      mfma_v(sa[0], a, kf[0][s]);
      mfma_v(sa[1], a, kf[1][s]);
    }
  }
#pragma unroll
  for (int s = 0; s < D / 16; ++s) {
    const bf16x8 a = row_read<D>(Ds, rb + l31, s, h);
    const bf16x8 v0 = *(lds_bf16x8*)(Vl + swzd<D>(l31, 2 * s + h));
    const bf16x8 v1 = *(lds_bf16x8*)(Vl + swzd<D>(32 + l31, 2 * s + h));
    if (s == 0) {
      mfma_v_first(dp[0], a, v0);
      mfma_v_first(dp[1], a, v1);
    } else {
      mfma_v(dp[0], a, v0);
      mfma_v(dp[1], a, v1);
    }
  }
  mfma_d_fence(sa, dp);
  // per-row softmax terms are read from LDS right where they are used (no 32-VGPR arrays)
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const f32x4 nl = *reinterpret_cast<const f32x4*>(NL + rb + 8 * g + 4 * h);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int e = 0; e < 4; ++e) sa[t][4 * g + e] = fast_exp2(__builtin_fmaf(sa[t][4 * g + e], sl2, nl[e]));
    }
  }
  if (MASK) {  // diagonal / tail slices only
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int mykey = key0 + 32 * t + l31;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int qi = qs0 + acc_row(i, h);
        if (qi >= S || mykey >= S || (CAUSAL && mykey > qi)) sa[t][i] = 0.f;
      }
    }
  }
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    const bf16x8 p0 = acc_to_b(sa[0], s2), p1 = acc_to_b(sa[1], s2);
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt) {
      const bf16x8 a = tr_read<D>(Ds, rb + 16 * s2 + 4 * h, dt, lane);
      dva[0][dt] = mfma(a, p0, dva[0][dt]);
      dva[1][dt] = mfma(a, p1, dva[1][dt]);
    }
  }
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const f32x4 dl = *reinterpret_cast<const f32x4*>(DL + rb + 8 * g + 4 * h);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int e = 0; e < 4; ++e) dp[t][4 * g + e] = sa[t][4 * g + e] * (dp[t][4 * g + e] - dl[e]);
    }
  }
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    const bf16x8 d0 = acc_to_b(dp[0], s2), d1 = acc_to_b(dp[1], s2);
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt) {
      const bf16x8 a = tr_read<D>(Qs, rb + 16 * s2 + 4 * h, dt, lane);
      dka[0][dt] = mfma(a, d0, dka[0][dt]);
      dka[1][dt] = mfma(a, d1, dka[1][dt]);
    }
  }
}

// fp32 variant of store_accT for the head-split partial sums
template <int ND>
__device__ __forceinline__ void store_accT_f32(float* rowp, const f32x16 (&acc)[ND], float mul, int h) {
#pragma unroll
  for (int dt = 0; dt < ND; ++dt) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      f32x4 w;
#pragma unroll
      for (int e = 0; e < 4; ++e) w[e] = acc[dt][4 * g + e] * mul;
      *reinterpret_cast<f32x4*>(rowp + dt * 32 + 8 * g + 4 * h) = w;
    }
  }
}

// Work balance.  A causal key block kb sees (nkb - kb) query tiles, so with one
// 256-key block per workgroup the first workgroup does twice the average work
// and sets the kernel time (measured: 2.97 ms vs 1.5 ms of balanced work at the
// 8k Llama shape).  Causal workgroups therefore process the pair of blocks
// {p, nkb-1-p} back to back (equal work per workgroup), and when that leaves
// fewer than ~2 workgroups per CU the GQA group's query heads are split over
// `gsplit` workgroups that write fp32 partials to `ws`, summed by
// attn_dkdv_reduce_kernel.
template <bool CAUSAL, int D, bool PF = false>
__global__ __launch_bounds__(256, 1) void attn_bwd_dkdv64_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    const bf16_t* __restrict__ dout, const float* __restrict__ lse, const float* __restrict__ delta,
    bf16_t* __restrict__ dk, bf16_t* __restrict__ dv, float* __restrict__ ws, int S, int H, int KV, int gsplit,
    float scale_log2, float scale, int64_t dkvs, int64_t kvs, int xcd) {
  constexpr int QT = 64;   // queries per staged tile
  constexpr int KW = 64;   // keys per wave
  constexpr int KB = 4 * KW;
  constexpr int TILE = 64 * 2 * D, STAGE = 2 * TILE;   // one 64-row Q (or dO, or V) tile; Q + dO
  // [Q|dO] x 2 stages (64 KiB at D 128), softmax row terms (1 KiB), this block's V rows per wave (4 tiles)
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE + 2 * 512 + 4 * TILE];
  int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  if (xcd) {
    // linear block L is dispatched to XCD L % 8: renumber so that each XCD runs whole (kv head,
    // batch) groups -- the workgroups that re-read one group's Q and dO then share an L2
    const int nx = gridDim.x, ny = gridDim.y;
    const int n = nx * ny * gridDim.z;
    const int L = bx + nx * (by + ny * bz);
    const int M = (L % 8) * (n / 8) + L / 8;
    bx = M % nx;
    by = (M / nx) % ny;
    bz = M / (nx * ny);
  }
  const int hk = by / gsplit, gs = by % gsplit, b = bz;
  const int lane = threadIdx.x & 63, h = lane >> 5, l31 = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // provably wave-uniform
  const int heads = (H / KV) / gsplit, hq0 = hk * (H / KV) + gs * heads;
  const int64_t qs = (int64_t)H * D, ks = kvs;   // q / dO rows contiguous; k / v rows kvs apart
  const int nkb = (S + KB - 1) / KB, nqt = (S + QT - 1) / QT;
  const int64_t nBHS = (int64_t)gridDim.z * H * S;  // delta = [delta | -lse*log2e]
  const DmaPlan<QT, 4, D> plan(qs, w, lane);
  const int blocks[2] = {bx, nkb - 1 - bx};
  const int nblocks = CAUSAL && blocks[1] != blocks[0] ? 2 : 1;
#pragma unroll 1
  for (int bi = 0; bi < nblocks; ++bi) {
    const int kb = blocks[bi];
    const int key0 = kb * KB + KW * w;   // first key of this wave
    // K stays in registers (B operand of S = Q K^T); V, the B operand of dP = dO V^T, goes to this
    // wave's LDS rows in the row_read layout: 64 fewer VGPRs for 16 more fragment reads per slice.
    char* Vw = smem + 2 * STAGE + 2 * 512 + w * TILE;
    bf16x8 kf[2][D / 16];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int64_t off = (int64_t)b * S * ks + (int64_t)min(key0 + 32 * t + l31, S - 1) * ks + hk * D;
#pragma unroll
      for (int s = 0; s < D / 16; ++s) {
        kf[t][s] = load_frag(k + off, s, h);
        *reinterpret_cast<bf16x8*>(Vw + swzd<D>(32 * t + l31, 2 * s + h)) = load_frag(v + off, s, h);
      }
    }
    f32x16 dka[2][D / 32], dva[2][D / 32];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int dt = 0; dt < D / 32; ++dt) {
        dka[t][dt] = f32x16{};
        dva[t][dt] = f32x16{};
      }
    }
    const int qt0 = CAUSAL ? (kb * KB) / QT : 0;
    const int per_head = nqt - qt0;
    const int total = per_head * heads;
    auto fetch = [&](int j, int st) {
      const int hq = hq0 + j / per_head;
      const int q0 = (qt0 + j % per_head) * QT;
      char* base = smem + st * STAGE;
      const int64_t off = (int64_t)b * S * qs + hq * D, nbytes = ((int64_t)S * qs - hq * D) * 2;
      const uint32_t soff = (uint32_t)(q0 * qs * 2);
      plan.issue(base, make_rsrc(q + off, nbytes), soff, w);
      plan.issue(base + TILE, make_rsrc(dout + off, nbytes), soff, w);
      float* lf = reinterpret_cast<float*>(smem + 2 * STAGE + st * 512);
      const int64_t row0 = ((int64_t)b * H + hq) * S;
      if (w == 0) dma_f32x64(lf, make_rsrc(delta + nBHS + row0, (int64_t)S * 4), q0, lane);
      if (w == 1) dma_f32x64(lf + QT, make_rsrc(delta + row0, (int64_t)S * 4), q0, lane);
    };
    if (total > 0) fetch(0, 0);
    wait_vm();
    __syncthreads();
    // Separate loops for the diagonal / tail tiles (masked body) and the rest (mask-free body):
    // one straight-line body per loop allocates registers far better than a branch per slice.
    auto run = [&](auto masked, int j0, int j1) {  // unrolled over the two stages (constant LDS offsets)
      constexpr bool MASK = decltype(masked)::value;
      auto step = [&](int j, auto stage) {
        constexpr int ST = decltype(stage)::value;   // == j & 1
        if (j + 1 < total) fetch(j + 1, 1 - ST);
        const char* Qs = smem + ST * STAGE;
        const char* Ds = Qs + TILE;
        const float* NL = reinterpret_cast<const float*>(smem + 2 * STAGE + ST * 512);
        const int q0 = (qt0 + j % per_head) * QT;
#pragma unroll 1
        for (int sub = 0; sub < QT / 32; ++sub) {
          const int qs0 = q0 + 32 * sub;
          if (CAUSAL && qs0 + 31 < key0) continue;  // wave-uniform: every key of the wave is after every query
          if constexpr (PF)
            dkdv64p_slice<MASK, CAUSAL, D>(Qs, Ds, NL, NL + QT, 32 * sub, kf, Vw, dka, dva, qs0, key0, S,
                                           scale_log2, lane);
          else
            dkdv64_slice<MASK, CAUSAL, D>(Qs, Ds, NL, NL + QT, 32 * sub, kf, Vw, dka, dva, qs0, key0, S, scale_log2,
                                          lane);
        }
        wait_vm();
        __syncthreads();   // also fences the LDS buffers before the next block's first fetch
      };
      int j = j0;
      if (j < j1 && (j & 1)) step(j++, std::integral_constant<int, 1>{});
#pragma unroll 1
      for (; j + 1 < j1; j += 2) {
        step(j, std::integral_constant<int, 0>{});
        step(j + 1, std::integral_constant<int, 1>{});
      }
      if (j < j1) step(j, std::integral_constant<int, 0>{});
    };
    // tiles [lo, hi) of every head need no mask for any wave of this workgroup
    int lo = CAUSAL ? min(KB / QT, per_head) : 0;
    int hi = max(lo, min(per_head, S / QT - qt0));
    if (kb * KB + KB > S) lo = hi = per_head;   // the block's keys run past S
#pragma unroll 1
    for (int hh = 0; hh < heads; ++hh) {
      const int base = hh * per_head;
      run(std::integral_constant<bool, true>{}, base, base + lo);
      run(std::integral_constant<bool, false>{}, base + lo, base + hi);
      run(std::integral_constant<bool, true>{}, base + hi, base + per_head);
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int mykey = key0 + 32 * t + l31;
      if (mykey >= S) continue;
      if (gsplit == 1) {
        store_accT(dk + ((int64_t)b * S + mykey) * dkvs + hk * D, dka[t], scale, h);
        store_accT(dv + ((int64_t)b * S + mykey) * dkvs + hk * D, dva[t], 1.f, h);
      } else {  // ws[gs][b][key][hk][dk|dv][D]
        float* row = ws + ((((int64_t)gs * gridDim.z + b) * S + mykey) * KV + hk) * 2 * D;
        store_accT_f32(row, dka[t], scale, h);
        store_accT_f32(row + D, dva[t], 1.f, h);
      }
    }
  }
}

// sum the head-split partials: ws[g][b][key][kv][2][HD] fp32 -> dk, dv bf16 (8 elements per thread)
template <int D>
__global__ __launch_bounds__(256) void attn_dkdv_reduce_kernel(const float* __restrict__ ws, bf16_t* __restrict__ dk,
                                                               bf16_t* __restrict__ dv, int64_t nrows, int gsplit,
                                                               int KV, int64_t dkvs) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;   // one 8-element chunk of a [2*D] row
  constexpr int CH = 2 * D / 8;
  if (i >= nrows * CH) return;
  const int64_t row = i / CH;
  const int c = (int)(i % CH);
  f32x4 a = {}, bq = {};
  for (int g = 0; g < gsplit; ++g) {
    const float* src = ws + ((int64_t)g * nrows + row) * 2 * D + 8 * c;
    a += *reinterpret_cast<const f32x4*>(src);
    bq += *reinterpret_cast<const f32x4*>(src + 4);
  }
  u32x4 o;
  o[0] = pack2(a[0], a[1]);
  o[1] = pack2(a[2], a[3]);
  o[2] = pack2(bq[0], bq[1]);
  o[3] = pack2(bq[2], bq[3]);
  // row = token * KV + kv head; dK / dV rows of a token are dkvs elements apart
  bf16_t* dst = (8 * c < D ? dk : dv) + (row / KV) * dkvs + (row % KV) * D + (8 * c) % D;
  *reinterpret_cast<u32x4*>(dst) = o;
}

// ---------------------------------------------------------------------------
// backward: dQ (a wave owns 32 queries; the forward's structure with
// dP^T = V dO^T and dQ^T += K^T dS^T)
// ---------------------------------------------------------------------------
template <bool MASK, bool CAUSAL, int D>
__device__ __forceinline__ void dq_tile(const char* Ks, const char* Vs, const bf16x8 (&qf)[D / 16],
                                        const bf16x8 (&df)[D / 16], f32x16 (&dqa)[D / 32], float nl2, float dl,
                                        int kv0, int qr, int S, float sl2, int lane) {
  const int h = lane >> 5, l31 = lane & 31;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    f32x16 st = f32x16{}, dpt = f32x16{};
#pragma unroll
    for (int s = 0; s < D / 16; ++s) st = mfma(row_read<D>(Ks, 32 * t + l31, s, h), qf[s], st);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < D / 16; ++s) dpt = mfma(row_read<D>(Vs, 32 * t + l31, s, h), df[s], dpt);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      float p = fast_exp2(__builtin_fmaf(st[i], sl2, nl2));
      if (MASK) {
        const int key = kv0 + 32 * t + acc_row(i, h);
        if (key >= S || (CAUSAL && key > qr)) p = 0.f;
      }
      dpt[i] = p * (dpt[i] - dl);  // dS^T
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const bf16x8 db = acc_to_b(dpt, s2);
#pragma unroll
      for (int dt = 0; dt < D / 32; ++dt)
        dqa[dt] = mfma(tr_read<D>(Ks, 32 * t + 16 * s2 + 4 * h, dt, lane), db, dqa[dt]);
    }
    // keep the scheduler from hoisting the next half's 32 LDS reads over this
    // one (that overlap costs ~100 registers and spills at 2 waves/SIMD)
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <bool CAUSAL, int D>
__global__ __launch_bounds__(256, 2) void attn_bwd_dq_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    const bf16_t* __restrict__ dout, const float* __restrict__ lse, const float* __restrict__ delta,
    bf16_t* __restrict__ dq, int S, int H, int KV, float scale_log2, float scale, int xcd, int64_t dqs,
    int64_t kvs) {
  constexpr int BQ = 128;
  constexpr int TILE = 64 * 2 * D, STAGE = 2 * TILE;
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  int qb, hq, b;
  grid_decode(xcd, H, KV, qb, hq, b);
  const int hk = hq / (H / KV);
  const int lane = threadIdx.x & 63, h = lane >> 5, l31 = lane & 31;
  const int w = threadIdx.x >> 6;
  const int q0 = qb * BQ;
  const int wq0 = q0 + 32 * w;
  const int64_t qs = (int64_t)H * D, ks = kvs;
  const bf16_t* kp = k + (int64_t)b * S * ks + hk * D;
  const bf16_t* vp = v + (int64_t)b * S * ks + hk * D;
  const int qr = wq0 + l31, qc = min(qr, S - 1);
  bf16x8 qf[D / 16], df[D / 16];
  {
    const bf16_t* qrow = q + (int64_t)b * S * qs + (int64_t)qc * qs + hq * D;
    const bf16_t* drow = dout + (int64_t)b * S * qs + (int64_t)qc * qs + hq * D;
#pragma unroll
    for (int s = 0; s < D / 16; ++s) {
      qf[s] = load_frag(qrow, s, h);
      df[s] = load_frag(drow, s, h);
    }
  }
  const int64_t nBHS = (int64_t)gridDim.z * H * S;  // delta = [delta | -lse*log2e]
  const float dl = delta[((int64_t)b * H + hq) * S + qc];
  const float nl2 = delta[nBHS + ((int64_t)b * H + hq) * S + qc];
  f32x16 dqa[D / 32];
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt) dqa[dt] = f32x16{};
  const int kv_end = CAUSAL ? min(S, q0 + BQ) : S;
  const int ntiles = (kv_end + 63) / 64;
  const DmaPlan<64, 4, D> plan(ks, w, lane);
  const int64_t kv_bytes = ((int64_t)S * ks - hk * D) * 2;
  const rsrc_t krs = make_rsrc(kp, kv_bytes), vrs = make_rsrc(vp, kv_bytes);
  const uint32_t tile_bytes = (uint32_t)(64 * ks * 2);
  plan.issue(smem, krs, 0, w);
  plan.issue(smem + TILE, vrs, 0, w);
  wait_vm();
  __syncthreads();
  const int nfull = CAUSAL ? min(q0, S) / 64 : S / 64;  // see the forward
  auto run = [&](auto masked, int it0, int it1) {  // unrolled over the two stages, as in the forward
    constexpr bool MASK = decltype(masked)::value;
    auto step = [&](int it, auto stage) {
      constexpr int ST = decltype(stage)::value;   // == it & 1
      const int kv0 = it * 64;
      if (it + 1 < ntiles) {
        plan.issue(smem + (1 - ST) * STAGE, krs, (it + 1) * tile_bytes, w);
        plan.issue(smem + (1 - ST) * STAGE + TILE, vrs, (it + 1) * tile_bytes, w);
      }
      const char* Ks = smem + ST * STAGE;
      if (!MASK || !CAUSAL || kv0 <= wq0 + 31)
        dq_tile<MASK, CAUSAL, D>(Ks, Ks + TILE, qf, df, dqa, nl2, dl, kv0, qr, S, scale_log2, lane);
      wait_vm();
      __syncthreads();
    };
    int it = it0;
    if (it < it1 && (it & 1)) step(it++, std::integral_constant<int, 1>{});
#pragma unroll 1
    for (; it + 1 < it1; it += 2) {
      step(it, std::integral_constant<int, 0>{});
      step(it + 1, std::integral_constant<int, 1>{});
    }
    if (it < it1) step(it, std::integral_constant<int, 0>{});
  };
  run(std::integral_constant<bool, false>{}, 0, nfull);
  run(std::integral_constant<bool, true>{}, nfull, ntiles);
  if (qr < S) store_accT(dq + ((int64_t)b * S + qr) * dqs + hq * D, dqa, scale, h);
}

}  // namespace

// XCD-aware work decode (grid_decode) for the forward and dQ kernels whenever every XCD
// can take whole K/V groups: -21 % kernel time each at B 2, S 8192, H 32, KV 8
// (profiles/r02_attn_xcd_ab.txt; the dK/dV kernel measured no gain from the same
// grouping and keeps its launch order).  EDL_ATTN_XCD=0 restores the launch order.
static int attn_xcd_map(int B, int KV) {
  const char* e = getenv("EDL_ATTN_XCD");
  const bool on = e == nullptr || atoi(e) != 0;
  return on && (B * KV) % 8 == 0 ? 1 : 0;
}

template <int D>
static void attn_fwd_launch(const void* q, const void* k, const void* v, void* o, float* lse, int B, int S, int H,
                            int KV, int causal, float sl2, int64_t qis, int64_t kvs, hipStream_t s) {
  dim3 grid((S + 127) / 128, H, B);
  const int xcd = attn_xcd_map(B, KV);
  if (causal)
    attn_fwd_kernel<true, D><<<grid, 256, 0, s>>>((const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v,
                                                      (bf16_t*)o, lse, S, H, KV, sl2, xcd, qis, kvs);
  else
    attn_fwd_kernel<false, D><<<grid, 256, 0, s>>>((const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v,
                                                       (bf16_t*)o, lse, S, H, KV, sl2, xcd, qis, kvs);
}

// dK/dV-64 work decomposition (see attn_bwd_dkdv64_kernel): returns gsplit, fills the grid
static int dkdv64_plan(int B, int S, int H, int KV, int causal, dim3* grid) {
  constexpr int kCUs = 256;   // MI355X: 8 XCDs x 32 CUs
  const int nkb = (S + 255) / 256, nx = causal ? (nkb + 1) / 2 : nkb, group = H / KV;
  int gsplit = 1;
  while ((int64_t)nx * KV * B * gsplit < kCUs && group % (2 * gsplit) == 0) gsplit *= 2;
  if (grid) *grid = dim3(nx, KV * gsplit, B);
  return gsplit;
}

static int dkdv_keys_per_wave() {
  static const int kpw = [] {
    const char* e = getenv("EDL_ATTN_DKDV");
    return e && atoi(e) == 32 ? 32 : 64;
  }();
  return kpw;
}

// delta: fp32 [2,B,H,S] scratch filled here (delta, -lse*log2(e)).
template <int D>
static int attn_bwd_impl(const void* q, const void* k, const void* v, const void* o, const void* dout,
                         const float* lse, float* delta, void* dq, void* dk, void* dv, float* ws, int B, int S, int H,
                         int KV, int causal, float scale, int64_t dqs, int64_t dkvs, int64_t kvs, hipStream_t s) {
  const int64_t nrows = (int64_t)B * S * H;
  attn_bwd_delta_kernel<D><<<(unsigned)((nrows * (D / 8) + 255) / 256), 256, 0, s>>>(
      (const bf16_t*)o, (const bf16_t*)dout, lse, delta, S, H, nrows);
  EDL_LAUNCH_CHECK();
  const float sl2 = scale * LOG2E;
  dim3 gkv((S + 127) / 128, KV, B), gq((S + 127) / 128, H, B);
  static const int occ = [] {
    const char* e = getenv("EDL_ATTN_DKDV_OCC");
    return e && atoi(e) == 2 ? 2 : 1;
  }();
  // head dim 64: the 32-keys-per-wave kernel fits two waves per SIMD and measured +7 % over the
  // 64-key one at the BERT-large shape (profiles/r02_attn_hd64_bert.txt); EDL_ATTN_DKDV=64 overrides
  static const bool force64 = [] {
    const char* e = getenv("EDL_ATTN_DKDV");
    return e && atoi(e) == 64;
  }();
  const int keys_per_wave = D == 128 ? dkdv_keys_per_wave() : (force64 ? 64 : 32);
  dim3 gkv64;
  const int gsplit = dkdv64_plan(B, S, H, KV, causal, &gkv64);
  static const int dkdv_xcd = [] {
    const char* e = getenv("EDL_ATTN_DKDV_XCD");
    return e ? atoi(e) : 0;
  }();
  const int xcd64 = dkdv_xcd && (gkv64.x * gkv64.y * gkv64.z) % 8 == 0 ? 1 : 0;
  const bf16_t *bq = (const bf16_t*)q, *bk = (const bf16_t*)k, *bv = (const bf16_t*)v, *bdo = (const bf16_t*)dout;
  static const bool dkdv_pf = [] {   // software-pipelined slices (dkdv64p_slice); EDL_ATTN_DKDV_PF=0: round 5's
    const char* e = getenv("EDL_ATTN_DKDV_PF");
    return !(e && atoi(e) == 0);
  }();
  if (keys_per_wave == 64) {
#define EDL_DKDV64(C, P)                                                                                    \
  attn_bwd_dkdv64_kernel<C, D, P><<<gkv64, 256, 0, s>>>(bq, bk, bv, bdo, lse, delta, (bf16_t*)dk, (bf16_t*)dv, \
                                                        ws, S, H, KV, gsplit, sl2, scale, dkvs, kvs, xcd64)
    if (causal) {
      if (dkdv_pf) EDL_DKDV64(true, true); else EDL_DKDV64(true, false);
    } else {
      if (dkdv_pf) EDL_DKDV64(false, true); else EDL_DKDV64(false, false);
    }
#undef EDL_DKDV64
    if (gsplit > 1) {
      EDL_LAUNCH_CHECK();
      const int64_t rows = (int64_t)B * S * KV;
      attn_dkdv_reduce_kernel<D><<<(unsigned)((rows * (2 * D / 8) + 255) / 256), 256, 0, s>>>(
          ws, (bf16_t*)dk, (bf16_t*)dv, rows, gsplit, KV, dkvs);
    }
  } else {
#define EDL_DKDV(C, O)                                                                                       \
  attn_bwd_dkdv_kernel<C, O, D><<<gkv, 256, 0, s>>>(bq, bk, bv, bdo, lse, delta, (bf16_t*)dk, (bf16_t*)dv, S, H, \
                                                    KV, sl2, scale, dkvs, kvs)
    if (causal) {
      if (occ == 2 || D == 64) EDL_DKDV(true, 2); else EDL_DKDV(true, 1);
    } else {
      if (occ == 2 || D == 64) EDL_DKDV(false, 2); else EDL_DKDV(false, 1);
    }
#undef EDL_DKDV
  }
  EDL_LAUNCH_CHECK();
  if (causal)
    attn_bwd_dq_kernel<true, D><<<gq, 256, 0, s>>>(bq, bk, bv, bdo, lse, delta, (bf16_t*)dq, S, H, KV, sl2, scale,
                                                   attn_xcd_map(B, KV), dqs, kvs);
  else
    attn_bwd_dq_kernel<false, D><<<gq, 256, 0, s>>>(bq, bk, bv, bdo, lse, delta, (bf16_t*)dq, S, H, KV, sl2, scale,
                                                    attn_xcd_map(B, KV), dqs, kvs);
  EDL_LAUNCH_CHECK();
  return 0;
}

extern "C" {

// input row strides: q rows qis (>= H*D) and k / v rows kvs (>= KV*D) elements apart, e.g. the
// q / k / v slices of one packed [B, S, 3, H, D] projection (BERT's fused qkv Linear: no split
// pass).  The LDS-DMA descriptors address a batch's S rows in 32 bits.
static bool strides_ok(int S, int H, int KV, int D, int64_t qis, int64_t kvs) {
  return qis >= (int64_t)H * D && kvs >= (int64_t)KV * D && qis % 8 == 0 && kvs % 8 == 0 &&
         (int64_t)S * kvs * 2 < (int64_t(1) << 32) && (int64_t)S * qis * 2 < (int64_t(1) << 32);
}

// head dim D = 64 or 128 (bf16, any S, GQA with H % KV == 0); o is written contiguous [B, S, H, D]
int edl_attn_fwd_strided(const void* q, const void* k, const void* v, void* o, float* lse, int B, int S, int H,
                         int KV, int D, int causal, float scale, int64_t qis, int64_t kvs, hipStream_t s) {
  if ((D != 64 && D != 128) || H % KV != 0 || S <= 0) return (int)hipErrorInvalidValue;
  if (!strides_ok(S, H, KV, D, qis, kvs)) return (int)hipErrorInvalidValue;
  const float sl2 = scale * LOG2E;
  // EDL_ATTN_FWD=64: the software-pipelined 64-queries-per-wave kernel (head dim 128)
  const char* sel = getenv("EDL_ATTN_FWD");
  if (D == 128 && sel && atoi(sel) == 64) {
    dim3 g64((S + 255) / 256, H, B);
    if (causal)
      attn_fwd64_kernel<true><<<g64, 256, 0, s>>>((const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v,
                                                     (bf16_t*)o, lse, S, H, KV, sl2, qis, kvs);
    else
      attn_fwd64_kernel<false><<<g64, 256, 0, s>>>((const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v,
                                                      (bf16_t*)o, lse, S, H, KV, sl2, qis, kvs);
    EDL_LAUNCH_CHECK();
    return 0;
  }
  if (D == 128)
    attn_fwd_launch<128>(q, k, v, o, lse, B, S, H, KV, causal, sl2, qis, kvs, s);
  else
    attn_fwd_launch<64>(q, k, v, o, lse, B, S, H, KV, causal, sl2, qis, kvs, s);
  EDL_LAUNCH_CHECK();
  return 0;
}

int edl_attn_fwd(const void* q, const void* k, const void* v, void* o, float* lse, int B, int S, int H, int KV,
                 int D, int causal, float scale, hipStream_t s) {
  return edl_attn_fwd_strided(q, k, v, o, lse, B, S, H, KV, D, causal, scale, (int64_t)H * D, (int64_t)KV * D, s);
}

// fp32 workspace the backward needs for the head-split dK/dV partials (0 = none); sized
// for head dim 128 (an upper bound for 64)
int64_t edl_attn_bwd_ws_bytes(int B, int S, int H, int KV, int causal) {
  if (KV <= 0 || H % KV != 0) return 0;
  const int g = dkdv64_plan(B, S, H, KV, causal, nullptr);
  return g == 1 ? 0 : (int64_t)g * B * S * KV * 2 * HD * 4;
}

// dq / dk / dv may be row-strided views: token rows dqs (>= H*D) and dkvs (>= KV*D) elements
// apart, e.g. the q / k / v slices of one packed [B, S, 3, H, D] gradient (BERT's fused
// qkv projection takes it without a concatenation pass).  Inputs: k / v rows kvs apart (the
// packed projection's slices); q, o and dout contiguous [B, S, H, D] (the dK/dV kernel stages
// q and dout tiles with one DMA plan).
int edl_attn_bwd_strided(const void* q, const void* k, const void* v, const void* o, const void* dout,
                         const float* lse, float* delta, void* dq, void* dk, void* dv, float* ws, int B, int S, int H,
                         int KV, int D, int causal, float scale, int64_t dqs, int64_t dkvs, int64_t kvs,
                         hipStream_t s) {
  if ((D != 64 && D != 128) || H % KV != 0 || S <= 0) return (int)hipErrorInvalidValue;
  if (dqs < (int64_t)H * D || dkvs < (int64_t)KV * D || dqs % 8 || dkvs % 8) return (int)hipErrorInvalidValue;
  if (!strides_ok(S, H, KV, D, (int64_t)H * D, kvs)) return (int)hipErrorInvalidValue;
  if (edl_attn_bwd_ws_bytes(B, S, H, KV, causal) > 0 && ws == nullptr) return (int)hipErrorInvalidValue;
  if (D == 128)
    return attn_bwd_impl<128>(q, k, v, o, dout, lse, delta, dq, dk, dv, ws, B, S, H, KV, causal, scale, dqs, dkvs,
                              kvs, s);
  return attn_bwd_impl<64>(q, k, v, o, dout, lse, delta, dq, dk, dv, ws, B, S, H, KV, causal, scale, dqs, dkvs, kvs,
                           s);
}

int edl_attn_bwd(const void* q, const void* k, const void* v, const void* o, const void* dout, const float* lse,
                 float* delta, void* dq, void* dk, void* dv, float* ws, int B, int S, int H, int KV, int D,
                 int causal, float scale, hipStream_t s) {
  return edl_attn_bwd_strided(q, k, v, o, dout, lse, delta, dq, dk, dv, ws, B, S, H, KV, D, causal, scale,
                              (int64_t)H * D, (int64_t)KV * D, (int64_t)KV * D, s);
}

}  // extern "C"
