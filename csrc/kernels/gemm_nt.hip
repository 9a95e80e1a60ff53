// bf16 "NT" GEMM for gfx950:  C[M, N] (+)= A[M, K] . B[N, K]^T   (A, B, C row-major,
// K contiguous in both operands; fp32 accumulation, bf16 C).
//
// Every big GEMM of the Llama training step has this form in easydl_amd's layouts
// (ops/fused.py): the forward Y = X W^T (A = X, B = W), the input gradient from the cached
// transposed weight dX = dY (W^T)^T (A = dY, B = W^T), and the weight gradient from the
// transposed activations the fused kernels emit dW += dY^T (X^T)^T (A = dY^T, B = X^T).
//
// Design (cdna_hip_programming.md §5 "Canonical CDNA GEMM", MI355X_MICROARCH.md):
//  * a 512-thread workgroup (8 waves, 2 x 4) owns a 256 x 256 block of C, one per CU
//    (LDS 2 x 64 KiB); a wave owns 128 (m) x 64 (n): 8 x 4 blocks of 16 x 16, 128 fp32
//    accumulator registers, v_mfma_f32_16x16x32_bf16 (the bf16 MFMA shape that holds the
//    higher clock on random data, MICROARCH "DVFS give-back" item 7);
//  * K tiles of 64 staged by LDS-DMA (buffer_load_dwordx4 ... lds, 16 B per lane): no
//    staging registers, no ds_write; two LDS stages, the next tile's DMA in flight under
//    the current tile's 64 MFMAs per wave, one barrier per tile;
//  * LDS rows are 128 B (64 bf16).  The DMA image is lane-linear, so the XOR swizzle goes
//    on the SOURCE address (rule 21): 16-B chunk c of row r sits at chunk c ^ swz(r),
//    swz(r) = ((r >> 1) & 7) ^ (((r >> 4) & 3) << 1) -- found by exhaustive search over
//    the ds_read_b128 lane groups of MICROARCH's LDS table: conflict-free for both
//    fragment read patterns below;
//  * operands swapped in the MFMA (D = B . A^T = C^T), with the 16 output rows of an MFMA
//    mapped to C columns 16 (i >> 2) + 4 nb + (i & 3): a lane's 4 x 4 results of one 16-row
//    block are 16 CONTIGUOUS columns of one row of C -> two 16-B stores, no LDS epilogue;
//  * tiles dealt to the 8 XCDs in contiguous runs (blocks b and b + 8 share an XCD; the
//    bijective form of §5 "XCD swizzle must be bijective"), and inside a run grouped
//    GROUP_M tile-rows deep, so the 32 workgroups an XCD runs at once share their A and B
//    K-tiles in that XCD's L2.
//
// Shapes: M, N multiples of 256, K a multiple of 64, 16-B aligned rows (checked on the
// host side, ops/gemm.py); anything else stays with hipBLASLt.
#include <type_traits>

#include "mfma_tile.h"

using namespace edl;
using namespace edl_tile;

namespace {

typedef float f32x4v __attribute__((ext_vector_type(4)));

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int ROWB = BK * 2;               // LDS bytes per tile row (8 chunks of 16 B: whole 128-B lines)
constexpr int TILE = 256 * ROWB;           // one operand's K-stage: 32 KiB
constexpr int NST = 2;                     // the next K-tile's DMA in flight under the one being read
// LDS: [A stages 0..1 | B stages 0..1]: every fragment read is a per-lane base register (one per
// operand and swizzle class) plus an immediate < 64 KiB (stage, row block)
constexpr int AOFF(int st) { return st * TILE; }
constexpr int BOFF(int st) { return NST * TILE + st * TILE; }

// chunk c of row r sits at chunk c ^ swz(r) (exhaustive search over the ds_read_b128 lane
// groups: conflict-free for both fragment read patterns of this kernel)
__device__ __forceinline__ int swz(int r) { return ((r >> 1) & 7) ^ (((r >> 4) & 3) << 1); }

__device__ __forceinline__ f32x4v mfma16(const bf16x8& a, const bf16x8& b, const f32x4v& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

typedef __attribute__((address_space(3))) char lds_c;
typedef __attribute__((address_space(3))) bf16x8 lds_frag_t;

__device__ __forceinline__ bf16x8 lds_frag(const lds_c* base, uint32_t off) {
  return *reinterpret_cast<const lds_frag_t*>(base + off);
}

// ACC: 0 = C = A B^T (bf16), 1 = C += A B^T (bf16 C read, fp32 add, bf16 store)
// DIAG: 1 = timing probe, no DMA after the prologue (compute + LDS reads only, wrong results);
//       2 = timing probe, DMA + waits + barriers only (no MFMA)
template <int ACC, int DIAG = 0>
__global__ __launch_bounds__(512, 1) void gemm_nt_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                                         bf16_t* __restrict__ C, int M, int N, int K, int lda,
                                                         int ldb, int ldc, int group_m) {
  __shared__ __attribute__((aligned(16))) char smem[2 * NST * TILE];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = w >> 2, wn = w & 3;
  // ---- tile assignment: XCD-contiguous runs, grouped GROUP_M tile-rows deep
  const int tm_n = M / BM, tn_n = N / BN;
  const int nwg = tm_n * tn_n;
  int wg = blockIdx.x;
  {
    const int q = nwg >> 3, r = nwg & 7, x = wg & 7;
    wg = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (wg >> 3);
  }
  const int width = group_m * tn_n;
  const int g = wg / width, first_m = g * group_m;
  const int gsize = min(tm_n - first_m, group_m);
  const int tm = first_m + (wg % width) % gsize, tn = (wg % width) / gsize;
  const int m0 = tm * BM, n0 = tn * BN;

  // ---- LDS-DMA plan: per operand and stage, wave w fills rows 32w .. 32w + 31 in four 1-KiB
  // pieces of 8 rows; lane l lands at row 32w + 8i + (l >> 3), physical chunk l & 7, so it
  // fetches logical chunk (l & 7) ^ swz(row)
  uint32_t va[4], vb[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = 32 * w + 8 * i + (lane >> 3);
    const int c = (lane & 7) ^ swz(r);
    va[i] = (uint32_t)(((int64_t)r * lda + 8 * c) * 2);
    vb[i] = (uint32_t)(((int64_t)r * ldb + 8 * c) * 2);
  }
  const rsrc_t ra = make_rsrc(A + (int64_t)m0 * lda, (uint32_t)(BM * (int64_t)lda * 2));
  const rsrc_t rb = make_rsrc(B + (int64_t)n0 * ldb, (uint32_t)(BN * (int64_t)ldb * 2));
  auto piece = [&](int kt, auto buf, auto pc) {
    constexpr int ST = decltype(buf)::value, P = decltype(pc)::value;
    const uint32_t soff = (uint32_t)(kt * BK * 2);
    if constexpr (P < 4) buffer_load_lds16(ra, smem + AOFF(ST) + (32 * w + 8 * P) * ROWB, va[P], soff);
    else buffer_load_lds16(rb, smem + BOFF(ST) + (32 * w + 8 * (P - 4)) * ROWB, vb[P - 4], soff);
  };
  auto issue = [&](int kt, auto buf) {
    piece(kt, buf, std::integral_constant<int, 0>{}); piece(kt, buf, std::integral_constant<int, 1>{});
    piece(kt, buf, std::integral_constant<int, 2>{}); piece(kt, buf, std::integral_constant<int, 3>{});
    piece(kt, buf, std::integral_constant<int, 4>{}); piece(kt, buf, std::integral_constant<int, 5>{});
    piece(kt, buf, std::integral_constant<int, 6>{}); piece(kt, buf, std::integral_constant<int, 7>{});
  };

  // ---- fragment read offsets (bytes within a stage; k-step kk adds 64 B = 4 chunks).  swz()
  // depends on row bits 1..5, so the XOR part of a fragment's chunk is per-lane XOR a constant
  // of the 16-row block: one base register per (block class, k-step), the block's row offset
  // goes in the instruction's immediate.
  // A-side operand (MFMA B input): row m = 128 wm + 16 mb + i (i = l & 15), chunk 4 kk + (l >> 4);
  //   swz = ((i >> 1) & 7) ^ ((mb & 3) << 1)
  // B-side operand (MFMA A input): row n = 64 wn + 16 (i >> 2) + 4 nb + (i & 3);
  //   swz = ((i >> 1) & 1) ^ (nb << 1) ^ ((i >> 2) << 1)
  uint32_t oa[4][2], ob[4][2];
  {
    const int i = lane & 15, q = lane >> 4;
#pragma unroll
    for (int c4 = 0; c4 < 4; ++c4) {
      const int ra_ = 128 * wm + i;
      const int rb_ = 64 * wn + 16 * (i >> 2) + (i & 3);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        oa[c4][kk] = (uint32_t)(AOFF(0) + ra_ * ROWB + (((4 * kk + q) ^ ((i >> 1) & 7) ^ (c4 << 1)) << 4));
        ob[c4][kk] = (uint32_t)(BOFF(0) + rb_ * ROWB +
                                (((4 * kk + q) ^ ((i >> 1) & 1) ^ (c4 << 1) ^ ((i >> 2) << 1)) << 4));
      }
    }
  }

  const lds_c* L = (const lds_c*)smem;
  f32x4v acc[8][4];
#pragma unroll
  for (int mb = 0; mb < 8; ++mb)
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) acc[mb][nb] = f32x4v{0.f, 0.f, 0.f, 0.f};

  const int nk = K / BK;
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  issue(0, S0{});
  auto step = [&](int kt, auto stage) {
    constexpr int ST = decltype(stage)::value;
    constexpr int SO = ST * TILE;   // stage offset inside the A and inside the B region
    // this wave's DMA of tile kt has landed; after the barrier every wave's has, and every
    // wave has finished reading the other stage (tile kt - 1): it may be refilled
    __builtin_amdgcn_s_waitcnt(0x0070);   // vmcnt(0) lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
    using NS = std::integral_constant<int, 1 - ST>;
    const bool more = kt + 1 < nk;
    if (more && DIAG != 1) issue(kt + 1, NS{});
    auto mma_row = [&](const bf16x8* fb, const bf16x8& fa, int mb) {
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) acc[mb][nb] = mfma16(fb[nb], fa, acc[mb][nb]);
    };
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 fa[8], fb[4];
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) fb[nb] = lds_frag(L + SO + 4 * nb * ROWB, ob[nb][kk]);
#pragma unroll
      for (int mb = 0; mb < 8; ++mb) fa[mb] = lds_frag(L + SO + 16 * mb * ROWB, oa[mb & 3][kk]);
      __builtin_amdgcn_s_setprio(1);
      if constexpr (DIAG == 2) {
        // DMA-only probe: fragment reads and MFMAs skipped, only the loads, waits and barriers
        if (fb[0][0] == 12345 && fa[0][0] == 54321) acc[0][0][0] += 1.f;
      } else {
#pragma unroll
        for (int mb = 0; mb < 8; ++mb) mma_row(fb, fa[mb], mb);
      }
      __builtin_amdgcn_s_setprio(0);
    }
  };
  int kt = 0;
#pragma unroll 1
  for (; kt + 1 < nk; kt += 2) {
    step(kt, S0{});
    step(kt + 1, S1{});
  }
  if (kt < nk) step(kt, S0{});

  // ---- epilogue: acc[mb][nb][r] = C[m][n], m = 128 wm + 16 mb + (l & 15),
  // n = 64 wn + 16 (l >> 4) + 4 nb + r  ->  16 contiguous columns per lane and row
  const int q = lane >> 4;
#pragma unroll
  for (int mb = 0; mb < 8; ++mb) {
    const int m = m0 + 128 * wm + 16 * mb + (lane & 15);
    bf16_t* p = C + (int64_t)m * ldc + n0 + 64 * wn + 16 * q;
    float v[16];
#pragma unroll
    for (int nb = 0; nb < 4; ++nb)
#pragma unroll
      for (int r = 0; r < 4; ++r) v[4 * nb + r] = acc[mb][nb][r];
    if (ACC) {
      const u32x4 o0 = reinterpret_cast<const u32x4*>(p)[0], o1 = reinterpret_cast<const u32x4*>(p)[1];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[2 * e] += bflo(o0[e]);
        v[2 * e + 1] += bfhi(o0[e]);
        v[8 + 2 * e] += bflo(o1[e]);
        v[8 + 2 * e + 1] += bfhi(o1[e]);
      }
    }
    u32x4 s0, s1;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      s0[e] = pack2(v[2 * e], v[2 * e + 1]);
      s1[e] = pack2(v[8 + 2 * e], v[8 + 2 * e + 1]);
    }
    reinterpret_cast<u32x4*>(p)[0] = s0;
    reinterpret_cast<u32x4*>(p)[1] = s1;
  }
}

}  // namespace

extern "C" {

// C (+)= A B^T; returns hipErrorInvalidValue for shapes the kernel does not take.
int edl_gemm_nt(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
                int accumulate, int group_m, hipStream_t stream) {
  if (M % BM || N % BN || K % BK || lda % 8 || ldb % 8 || ldc % 8 || M <= 0 || N <= 0 || K <= 0)
    return (int)hipErrorInvalidValue;
  if ((int64_t)BM * lda * 2 >= (1ll << 32) || (int64_t)BN * ldb * 2 >= (1ll << 32))
    return (int)hipErrorInvalidValue;
  if (group_m <= 0) group_m = 8;
  const int nwg = (M / BM) * (N / BN);
  if (accumulate)
    gemm_nt_kernel<1><<<nwg, 512, 0, stream>>>((const bf16_t*)A, (const bf16_t*)B, (bf16_t*)C, M, N, K, lda, ldb,
                                               ldc, group_m);
  else
    gemm_nt_kernel<0><<<nwg, 512, 0, stream>>>((const bf16_t*)A, (const bf16_t*)B, (bf16_t*)C, M, N, K, lda, ldb,
                                               ldc, group_m);
  EDL_LAUNCH_CHECK();
  return 0;
}

// timing probes of the kernel's parts (see DIAG); results are garbage
int edl_gemm_nt_diag(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
                     int mode, int group_m, hipStream_t stream) {
  if (M % BM || N % BN || K % BK) return (int)hipErrorInvalidValue;
  const int nwg = (M / BM) * (N / BN);
  if (mode == 1)
    gemm_nt_kernel<0, 1><<<nwg, 512, 0, stream>>>((const bf16_t*)A, (const bf16_t*)B, (bf16_t*)C, M, N, K, lda, ldb,
                                                  ldc, group_m);
  else if (mode == 2)
    gemm_nt_kernel<0, 2><<<nwg, 512, 0, stream>>>((const bf16_t*)A, (const bf16_t*)B, (bf16_t*)C, M, N, K, lda, ldb,
                                                  ldc, group_m);
  else
    return (int)hipErrorInvalidValue;
  EDL_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
