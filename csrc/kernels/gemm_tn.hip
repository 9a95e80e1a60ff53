// Weight-gradient GEMM in the layouts the backward already holds (gfx950, bf16 in,
// fp32 accumulate, v_mfma_f32_32x32x16_bf16).
//
//   C[N, J] (+)= A^T B,   A = dY [M, N],  B = X [M, J],  both row-major, M = tokens
//
// hipBLASLt runs this "TN" form 15-35 % slower than its NT form, so until now the
// backward transposed dY and X first (two LDS-tiled transposes per linear layer,
// ~2 % of the Llama-3-8B step and ~7 % of BERT-large's).  Here the reduction axis M
// is the ROW axis of both operands: a [32 rows][128 columns] tile of each is staged
// into LDS as stored (LDS-DMA, buffer_load ... lds, 256-B rows with the XOR swizzle
// of mfma_tile.h) and both MFMA operands are read from it with ds_read_b64_tr_b16,
// the transposing LDS read -- the layout change costs nothing beyond the reads the
// MFMAs need anyway.  No transposed copies are ever written.
//
// Tiling: a workgroup (4 waves) owns a 128 (n) x 256 (j) block of C; wave (wn, wj)
// owns 64 x 128 = 2 x 4 blocks of 32 x 32 (8 accumulators, 128 registers), so each k-step
// of 16 reads 2 A + 4 B fragments for 8 MFMAs.  32-row k-stages, three LDS stages
// (72 KiB) filled two stages ahead, one barrier per stage; two workgroups per CU.
// Weight gradients of small layers have few C tiles against a deep M (BERT-large:
// 1024 x 1024 outputs = 32 tiles, M = 16384): M is then split over workgroups
// (fp32 partial slab + one reduce pass) so the launch fills the 256 CUs; hipBLASLt
// ran those at 0.6-1.0 PF/s with small tiles.  Work ids are dealt so that each XCD
// gets a contiguous run of tiles (blocks b and b+8 share an XCD): tiles sharing A
// columns share that XCD's L2.
//
// Capability source: SURVEY.md §2.4 (fused hot ops of the training step), VERDICT r02
// "remove standalone transposes".
#include <cstdlib>
#include <type_traits>

#include "mfma_tile.h"

using namespace edl;
using namespace edl_tile;

namespace {

constexpr int BN = 128, BJ = 256, KS = 32, NST = 3;
constexpr int TILE = KS * 256;   // one [32][128] bf16 tile = 8 KiB
constexpr int STAGE = 3 * TILE;  // A tile + two B tiles
constexpr int kCUs = 256;

// ds_read_b64_tr_b16 as inline asm.  With the builtin, hipcc's wait-count pass does not
// prove the transposing read disjoint from the in-flight LDS-DMA and emits vmcnt(0)
// before the first read of every stage, draining the prefetch (the .s showed it; the
// plain ds_read_b128 row reads of attention.hip escape it).  The asm read is invisible to
// that pass, so the kernel orders it itself: reads follow the barrier that publishes
// their stage, and lgkm_wait() ties the fragments to an explicit lgkmcnt wait.
template <int OFF>
__device__ __forceinline__ i16x4 ds_tr(uint32_t addr) {
  i16x4 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
  return r;
}
template <int OFF>
__device__ __forceinline__ bf16x8 frag_tr(uint32_t lo, uint32_t hi) {
  const i16x8 v = __builtin_shufflevector(ds_tr<OFF>(lo), ds_tr<OFF>(hi), 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}
// wait until at most N LDS reads are outstanding; the fragments pass through the asm so
// no MFMA that reads them can be scheduled above the wait
template <int N>
__device__ __forceinline__ void lgkm_wait(bf16x8& a0, bf16x8& a1, bf16x8& b0, bf16x8& b1, bf16x8& b2, bf16x8& b3) {
  asm volatile("s_waitcnt lgkmcnt(%6)" : "+v"(a0), "+v"(a1), "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3) : "i"(N));
}

// OUT: 0 = bf16 C, 1 = fp32 C, 2 = fp32 partial slab [splits][N][J]
template <int OUT>
__global__ __launch_bounds__(256, 2) void gemm_tn_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                                         void* __restrict__ C, int M, int N, int J, int mchunk,
                                                         int accumulate) {
  __shared__ __attribute__((aligned(16))) char smem[NST * STAGE];
  const int lane = threadIdx.x & 63, h = lane >> 5, l31 = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wn = w >> 1, wj = w & 1;
  const int tjn = J / BJ, T = (N / BN) * tjn;
  const int W = gridDim.x;
  int id = blockIdx.x;
  if ((W & 7) == 0) id = (id & 7) * (W >> 3) + (id >> 3);   // contiguous work per XCD
  const int s = id / T, t = id % T;
  const int n0 = (t / tjn) * BN, j0 = (t % tjn) * BJ;
  const int m_begin = s * mchunk, m_end = min(M, m_begin + mchunk);
  const int nk = (m_end - m_begin + KS - 1) / KS;
  const DmaPlan<KS, 4> pa(N, w, lane), pb(J, w, lane);
  // loop-invariant LDS byte addresses of this lane's transposed fragment reads (k-step 0 of
  // stage 0; stage and k-step offsets go in the immediate).  The MFMA operand with rows =
  // tile columns 32*dt .. 32*dt+31 (lane & 31) and k = tile rows kb.. comes from two
  // ds_read_b64_tr_b16 at rows kb + qq and kb + 8 + qq (qq = (lane & 15) >> 2, kb = 4h),
  // element j <-> k row kb + 8*(j>>2) + (j&3): two operands read with the same kb pair the
  // same k in every element, so their MFMA sums over 16 tile rows.  wj's B half is folded in.
  uint32_t alo[2], ahi[2], blo[4], bhi[4];
  {
    const uint32_t base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
    const int i = lane & 15, qq = i >> 2, p = i & 3;
    auto addr = [&](int row, int dt) {
      const int col = dt * 32 + ((lane >> 4) & 1) * 16 + 4 * p;
      return base + (uint32_t)(swz(row, col >> 3) + ((col >> 2) & 1) * 8);
    };
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      alo[q] = addr(4 * h + qq, 2 * wn + q);
      ahi[q] = addr(4 * h + 8 + qq, 2 * wn + q);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      blo[q] = addr(4 * h + qq, q) + wj * TILE;
      bhi[q] = addr(4 * h + 8 + qq, q) + wj * TILE;
    }
  }

  // stage buffer `BUF` (a template constant, so the LDS-DMA targets and the LDS reads of
  // different stages sit at provably different constant offsets of smem and the
  // compiler's wait-count pass does not drain the in-flight DMA before every read)
  auto issue = [&](int it, auto buf) {
    constexpr int BUF = decltype(buf)::value;
    const int m0 = m_begin + it * KS;
    const uint32_t rows = (uint32_t)min(KS, m_end - m0);   // rows past the chunk read as zeros
    char* st = smem + BUF * STAGE;
    pa.issue(st, make_rsrc(A + (int64_t)m0 * N + n0, rows * (uint32_t)N * 2), w);
    const bf16_t* bp = B + (int64_t)m0 * J + j0;
    pb.issue(st + TILE, make_rsrc(bp, rows * (uint32_t)J * 2), w);
    pb.issue(st + 2 * TILE, make_rsrc(bp + 128, rows * (uint32_t)J * 2 - 256), w);
  };

  f32x16 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) acc[i][jj] = f32x16{};
  }
  using C0 = std::integral_constant<int, 0>;
  using C1 = std::integral_constant<int, 1>;
  using C2 = std::integral_constant<int, 2>;
  if (nk > 0) issue(0, C0{});
  if (nk > 1) issue(1, C1{});
  auto step = [&](int it, auto stage) {
    constexpr int ST = decltype(stage)::value;   // == it % NST
    // this wave's pieces of stage `it` have landed (stage it+1's 6 may still fly), its LDS
    // reads of stage it-1 are done; after the barrier the same holds for every wave, so
    // stage it is complete in LDS and stage it-1's buffer may be refilled
    if (it + 1 < nk)
      __builtin_amdgcn_s_waitcnt(0x0076);   // vmcnt(6) lgkmcnt(0)
    else
      __builtin_amdgcn_s_waitcnt(0x0070);   // vmcnt(0) lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
    if (it + 2 < nk) issue(it + 2, std::integral_constant<int, (ST + 2) % NST>{});
    // 2 k-steps x (2 A + 4 B fragments) = 24 reads issued back to back; the first k-step's
    // MFMAs start once its 12 have returned (LDS returns in order)
    constexpr int SO = ST * STAGE;
    bf16x8 f[2][6];   // [k-step][A blocks 2wn, 2wn+1 | B blocks 0..3 of this wave's 128 columns]
#pragma unroll
    for (int q = 0; q < 2; ++q) f[0][q] = frag_tr<SO>(alo[q], ahi[q]);
#pragma unroll
    for (int q = 0; q < 4; ++q) f[0][2 + q] = frag_tr<SO + TILE>(blo[q], bhi[q]);
#pragma unroll
    for (int q = 0; q < 2; ++q) f[1][q] = frag_tr<SO + 16 * 256>(alo[q], ahi[q]);
#pragma unroll
    for (int q = 0; q < 4; ++q) f[1][2 + q] = frag_tr<SO + TILE + 16 * 256>(blo[q], bhi[q]);
    lgkm_wait<12>(f[0][0], f[0][1], f[0][2], f[0][3], f[0][4], f[0][5]);
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      acc[0][jj] = mfma(f[0][0], f[0][2 + jj], acc[0][jj]);
      acc[1][jj] = mfma(f[0][1], f[0][2 + jj], acc[1][jj]);
    }
    __builtin_amdgcn_sched_barrier(0);   // k-step 1's wait stays behind k-step 0's MFMAs
    lgkm_wait<0>(f[1][0], f[1][1], f[1][2], f[1][3], f[1][4], f[1][5]);
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      acc[0][jj] = mfma(f[1][0], f[1][2 + jj], acc[0][jj]);
      acc[1][jj] = mfma(f[1][1], f[1][2 + jj], acc[1][jj]);
    }
    __builtin_amdgcn_sched_barrier(0);   // the next stage's barrier stays behind these MFMAs
  };
  int it = 0;
#pragma unroll 1
  for (; it + 2 < nk; it += 3) {
    step(it, C0{});
    step(it + 1, C1{});
    step(it + 2, C2{});
  }
  if (it < nk) step(it++, C0{});
  if (it < nk) step(it, C1{});
  // epilogue: accumulator register r of block (i, jj) is C[n][j] with
  // n = block row acc_row(r, h), j = block column lane & 31 (32 lanes = 32 consecutive j)
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int j = j0 + wj * 128 + jj * 32 + l31;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int n = n0 + wn * 64 + i * 32 + acc_row(r, h);
        const float v = acc[i][jj][r];
        if (OUT == 2) {
          reinterpret_cast<float*>(C)[((int64_t)s * N + n) * J + j] = v;
        } else if (OUT == 1) {
          float* p = reinterpret_cast<float*>(C) + (int64_t)n * J + j;
          *p = accumulate ? *p + v : v;
        } else {
          bf16_t* p = reinterpret_cast<bf16_t*>(C) + (int64_t)n * J + j;
          *p = f2bf(accumulate ? bf2f(*p) + v : v);
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// 256 x 256 tiles for weights big enough to fill the chip without splitting M (the
// Llama-3-8B projections: 384-1792 tiles).  One workgroup of 8 waves per CU, two per
// SIMD: wave (wn, wj) owns 128 (n) x 64 (j) = 4 x 2 blocks (128 accumulators), a k-step
// of 16 reads 4 A + 2 B fragments for 8 MFMAs.  A 4-wave form (128 x 128 per wave, one
// wave per SIMD) ran at 42 % MFMA busy, issue-bound on its LDS-DMA pieces and waits with
// nothing to hide them (PMC, profiles/r03_gemm_tn_ab.md); with two waves per SIMD one
// wave's DMA issue and waits run under the other's MFMAs (gate/up 3.85 -> 3.35 ms).
// Four 32 KiB LDS stages: the DMA of stage it+2 is issued at the top of stage it into
// the buffer stage it-2 used (every wave finished it before the previous barrier), and
// the transposed reads run one k-step ahead of the MFMAs across the barrier: k-step 1's
// reads are issued before k-step 0's MFMAs, and the next stage's k-step 0 reads right
// after the barrier that publishes it, before k-step 1's MFMAs.
// Tiles are visited in groups of 8 n-rows (j within the group, then the next group),
// each XCD taking a contiguous range: the ~32 workgroups an XCD runs at once share
// 8 A column blocks and 4 B column blocks in its L2.
// ---------------------------------------------------------------------------
constexpr int B2 = 256, STAGE2 = 4 * TILE, NB2 = 4;

template <int N6>
__device__ __forceinline__ void lgkm_wait6(bf16x8 (&f)[6]) {
  asm volatile("s_waitcnt lgkmcnt(%6)" : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]), "+v"(f[4]), "+v"(f[5])
               : "i"(N6));
}

template <int OUT>   // 0 = bf16 C, 1 = fp32 C
__global__ __launch_bounds__(512, 1) void gemm_tn256_kernel(const bf16_t* __restrict__ A,
                                                            const bf16_t* __restrict__ B, void* __restrict__ C,
                                                            int M, int N, int J, int accumulate) {
  __shared__ __attribute__((aligned(16))) char smem[NB2 * STAGE2];
  const int lane = threadIdx.x & 63, h = lane >> 5, l31 = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wn = w >> 2, wj = w & 3;
  const int tnn = N / B2, tjn = J / B2, T = tnn * tjn;
  int t = blockIdx.x;
  {   // contiguous range per XCD (bijective for any T: the first T % 8 XCDs get one more)
    const int q = T / 8, r = T % 8, x = t % 8, k = t / 8;
    t = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + k;
  }
  constexpr int GROUP = 8;
  const int g = t / (GROUP * tjn), rows_g = min(GROUP, tnn - g * GROUP), within = t - g * GROUP * tjn;
  const int n0 = (g * GROUP + within % rows_g) * B2, j0 = (within / rows_g) * B2;
  const int nk = (M + KS - 1) / KS;
  const DmaPlan<KS, 8> pa(N, w, lane), pb(J, w, lane);
  uint32_t alo[4], ahi[4], blo[2], bhi[2];   // this lane's fragment addresses, stage 0, k-step 0
  {
    const uint32_t base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
    const int i = lane & 15, qq = i >> 2, p = i & 3;
    auto addr = [&](int row, int dt) {
      const int col = dt * 32 + ((lane >> 4) & 1) * 16 + 4 * p;
      return base + (uint32_t)(swz(row, col >> 3) + ((col >> 2) & 1) * 8);
    };
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      alo[q] = addr(4 * h + qq, q) + wn * TILE;
      ahi[q] = addr(4 * h + 8 + qq, q) + wn * TILE;
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      blo[q] = addr(4 * h + qq, (wj & 1) * 2 + q) + (2 + (wj >> 1)) * TILE;
      bhi[q] = addr(4 * h + 8 + qq, (wj & 1) * 2 + q) + (2 + (wj >> 1)) * TILE;
    }
  }
  auto dma = [&](int it, int buf) {
    const int m0 = it * KS;
    const uint32_t rows = (uint32_t)min(KS, M - m0);
    char* st = smem + buf * STAGE2;
    const bf16_t* ap = A + (int64_t)m0 * N + n0;
    const bf16_t* bp = B + (int64_t)m0 * J + j0;
    pa.issue(st, make_rsrc(ap, rows * (uint32_t)N * 2), w);
    pa.issue(st + TILE, make_rsrc(ap + 128, rows * (uint32_t)N * 2 - 256), w);
    pb.issue(st + 2 * TILE, make_rsrc(bp, rows * (uint32_t)J * 2), w);
    pb.issue(st + 3 * TILE, make_rsrc(bp + 128, rows * (uint32_t)J * 2 - 256), w);
  };
  // the 6 fragments of k-step KSTEP of the stage in buffer `buf`: A blocks 0..3, B blocks 0..1
  auto reads = [&](bf16x8 (&f)[6], int buf, auto kstep) {
    constexpr int KO = decltype(kstep)::value * 16 * 256;
    const uint32_t bo = (uint32_t)buf * STAGE2;
#pragma unroll
    for (int q = 0; q < 4; ++q) f[q] = frag_tr<KO>(alo[q] + bo, ahi[q] + bo);
#pragma unroll
    for (int q = 0; q < 2; ++q) f[4 + q] = frag_tr<KO>(blo[q] + bo, bhi[q] + bo);
  };
  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) acc[i][jj] = f32x16{};
  }
  auto mmas = [&](const bf16x8 (&f)[6]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) acc[i][jj] = mfma(f[i], f[4 + jj], acc[i][jj]);
    }
  };
  using K0 = std::integral_constant<int, 0>;
  using K1 = std::integral_constant<int, 1>;
  bf16x8 cur[6], nxt[6];
  if (nk > 0) dma(0, 0);
  if (nk > 1) dma(1, 1);
  if (nk > 1)
    __builtin_amdgcn_s_waitcnt(0x0074);   // vmcnt(4): stage 0 landed (stage 1 may fly)
  else
    __builtin_amdgcn_s_waitcnt(0x0070);
  __builtin_amdgcn_s_barrier();
  if (nk > 0) reads(cur, 0, K0{});
#pragma unroll 1
  for (int it = 0; it < nk; ++it) {
    const int buf = it & 3;
    if (it + 2 < nk) dma(it + 2, (it + 2) & 3);
    lgkm_wait6<0>(cur);                    // k-step 0 of stage it
    reads(nxt, buf, K1{});                 // k-step 1 reads fly under k-step 0's MFMAs
    __builtin_amdgcn_sched_barrier(0);
    mmas(cur);
    __builtin_amdgcn_sched_barrier(0);
    if (it + 1 < nk) {
      if (it + 2 < nk)
        __builtin_amdgcn_s_waitcnt(0x0074);   // vmcnt(4): stage it+1 landed (it+2 may fly)
      else
        __builtin_amdgcn_s_waitcnt(0x0070);
      __builtin_amdgcn_s_barrier();           // ... in every wave: stage it+1 is readable
      reads(cur, (it + 1) & 3, K0{});         // next stage's k-step 0 under k-step 1's MFMAs
      lgkm_wait6<12>(nxt);
    } else {
      lgkm_wait6<0>(nxt);
    }
    __builtin_amdgcn_sched_barrier(0);
    mmas(nxt);
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int j = j0 + wj * 64 + jj * 32 + l31;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int n = n0 + wn * 128 + i * 32 + acc_row(r, h);
        const float v = acc[i][jj][r];
        if (OUT == 1) {
          float* p = reinterpret_cast<float*>(C) + (int64_t)n * J + j;
          *p = accumulate ? *p + v : v;
        } else {
          bf16_t* p = reinterpret_cast<bf16_t*>(C) + (int64_t)n * J + j;
          *p = f2bf(accumulate ? bf2f(*p) + v : v);
        }
      }
    }
  }
}

// C[i] (+)= sum_s slab[s][i], 8 elements per thread (N*J % 8 == 0)
__global__ __launch_bounds__(256) void gemm_tn_reduce_kernel(const float* __restrict__ slab, void* __restrict__ C,
                                                             int64_t n, int splits, int out_fp32, int accumulate) {
  const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;
  if (i >= n) return;
  f32x4 a = *reinterpret_cast<const f32x4*>(slab + i), b = *reinterpret_cast<const f32x4*>(slab + i + 4);
  for (int s = 1; s < splits; ++s) {
    a += *reinterpret_cast<const f32x4*>(slab + s * n + i);
    b += *reinterpret_cast<const f32x4*>(slab + s * n + i + 4);
  }
  if (out_fp32) {
    f32x4* o = reinterpret_cast<f32x4*>(reinterpret_cast<float*>(C) + i);
    if (accumulate) {
      a += o[0];
      b += o[1];
    }
    o[0] = a;
    o[1] = b;
  } else {
    u32x4* o = reinterpret_cast<u32x4*>(reinterpret_cast<bf16_t*>(C) + i);
    float f[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
    if (accumulate) {
      float old[8];
      unpack8(*o, old);
#pragma unroll
      for (int k = 0; k < 8; ++k) f[k] += old[k];
    }
    *o = pack8(f);
  }
}

// [G, N] fp32 column-sum partials of a bf16 [M, N] matrix: partial[g] sums rows r = g (mod G);
// the bias gradient of a linear layer whose weight gradient no longer passes dY through a
// transpose kernel.
// A block = CL column lanes (8 columns each) x RL row lanes (RL = 256 / CL, so narrow
// matrices still fill the block), 8 independent 16-B loads in flight per lane; the row
// lanes are combined through LDS.  (The one-row-lane, 4-deep form was latency-bound:
// 11.4 us for a BERT-large [16384, 1024] gradient, 73 calls per step.)
template <int RL>
__global__ __launch_bounds__(256) void colsum_bf16_partial_kernel(const bf16_t* __restrict__ x, int M, int N,
                                                                  float* __restrict__ partial, int G) {
  constexpr int CL = 256 / RL, U = 8;
  const int cl = threadIdx.x % CL, rl = threadIdx.x / CL;
  const int c = (blockIdx.x * CL + cl) * 8;
  const int g = blockIdx.y;
  float s[8] = {};
  if (c < N) {
    const int step = G * RL;
    int r = g + G * rl;
    for (; r + (U - 1) * step < M; r += U * step) {
      u32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = *reinterpret_cast<const u32x4*>(x + (int64_t)(r + u * step) * N + c);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        float f[8];
        unpack8(v[u], f);
#pragma unroll
        for (int k = 0; k < 8; ++k) s[k] += f[k];
      }
    }
    for (; r < M; r += step) {
      float f[8];
      unpack8(*reinterpret_cast<const u32x4*>(x + (int64_t)r * N + c), f);
#pragma unroll
      for (int k = 0; k < 8; ++k) s[k] += f[k];
    }
  }
  if (RL > 1) {
    __shared__ f32x4 red[RL > 1 ? RL - 1 : 1][CL][2];
    if (rl > 0) {
      red[rl - 1][cl][0] = f32x4{s[0], s[1], s[2], s[3]};
      red[rl - 1][cl][1] = f32x4{s[4], s[5], s[6], s[7]};
    }
    __syncthreads();
    if (rl > 0) return;
#pragma unroll
    for (int i = 0; i < RL - 1; ++i) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        s[k] += red[i][cl][0][k];
        s[4 + k] += red[i][cl][1][k];
      }
    }
  }
  if (c >= N) return;
  f32x4* o = reinterpret_cast<f32x4*>(partial + (int64_t)g * N + c);
  o[0] = f32x4{s[0], s[1], s[2], s[3]};
  o[1] = f32x4{s[4], s[5], s[6], s[7]};
}

}  // namespace

extern "C" {

// M-splits the TN weight-gradient GEMM uses for this shape (1 = no partial slab): enough
// work ids for ~one workgroup per CU, each split at least 1024 rows deep.
int edl_gemm_tn_splits(int M, int N, int J) {
  if (N <= 0 || J <= 0 || N % BN || J % BJ) return 0;
  static const int target = [] {   // work ids to aim for (EDL_GEMM_TN_WGS, default two per CU)
    const char* e = getenv("EDL_GEMM_TN_WGS");
    return e && atoi(e) > 0 ? atoi(e) : 2 * kCUs;
  }();
  const int T = (N / BN) * (J / BJ);
  int s = 1;
  while (T * s * 2 <= target && M / (2 * s) >= 1024 && s < 16) s *= 2;
  return s;
}

static bool use_tn256(int N, int J);

int64_t edl_gemm_tn_ws_bytes(int M, int N, int J) {
  if (use_tn256(N, J)) return 0;
  const int s = edl_gemm_tn_splits(M, N, J);
  return s > 1 ? (int64_t)s * N * J * 4 : 0;
}

// C[N, J] (+)= A^T B for row-major bf16 A [M, N], B [M, J]; C bf16 or fp32 (out_fp32),
// overwritten or accumulated into.  N % 128 == 0, J % 256 == 0, 16-B aligned rows;
// ws: fp32 scratch of edl_gemm_tn_ws_bytes (may be null when that is 0).
// the 256 x 256 kernel when it alone gives every CU a tile (no M split needed)
static bool use_tn256(int N, int J) {
  static const int mode = [] {
    const char* e = getenv("EDL_GEMM_TN256");
    return e ? atoi(e) : 1;
  }();
  return mode != 0 && N % B2 == 0 && J % B2 == 0 && (N / B2) * (J / B2) >= kCUs;
}

int edl_gemm_tn(const void* A, const void* B, void* C, int M, int N, int J, int out_fp32, int accumulate, float* ws,
                hipStream_t s) {
  if (M > 0 && use_tn256(N, J)) {
    if ((int64_t)32 * N * 2 >= (1ll << 32) || (int64_t)32 * J * 2 >= (1ll << 32)) return (int)hipErrorInvalidValue;
    const dim3 grid((N / B2) * (J / B2));
    if (out_fp32)
      gemm_tn256_kernel<1><<<grid, 512, 0, s>>>((const bf16_t*)A, (const bf16_t*)B, C, M, N, J, accumulate);
    else
      gemm_tn256_kernel<0><<<grid, 512, 0, s>>>((const bf16_t*)A, (const bf16_t*)B, C, M, N, J, accumulate);
    EDL_LAUNCH_CHECK();
    return 0;
  }
  const int splits = edl_gemm_tn_splits(M, N, J);
  if (splits <= 0 || M <= 0 || (splits > 1 && ws == nullptr)) return (int)hipErrorInvalidValue;
  if ((int64_t)32 * N * 2 >= (1ll << 32) || (int64_t)32 * J * 2 >= (1ll << 32)) return (int)hipErrorInvalidValue;
  const int T = (N / BN) * (J / BJ);
  const int mchunk = splits == 1 ? M : ((M + splits - 1) / splits + KS - 1) / KS * KS;
  const dim3 grid(T * splits);
  const bf16_t *a = (const bf16_t*)A, *b = (const bf16_t*)B;
  if (splits > 1) {
    gemm_tn_kernel<2><<<grid, 256, 0, s>>>(a, b, ws, M, N, J, mchunk, 0);
    EDL_LAUNCH_CHECK();
    const int64_t n = (int64_t)N * J;
    gemm_tn_reduce_kernel<<<(unsigned)((n / 8 + 255) / 256), 256, 0, s>>>(ws, C, n, splits, out_fp32, accumulate);
  } else if (out_fp32) {
    gemm_tn_kernel<1><<<grid, 256, 0, s>>>(a, b, C, M, N, J, mchunk, accumulate);
  } else {
    gemm_tn_kernel<0><<<grid, 256, 0, s>>>(a, b, C, M, N, J, mchunk, accumulate);
  }
  EDL_LAUNCH_CHECK();
  return 0;
}

int edl_colsum_bf16_groups(int M) { return M >= 64 * 256 ? 256 : (M >= 64 ? M / 64 : 1); }

// [G, N] fp32 column-sum partials of a bf16 [M, N] matrix (N % 8 == 0); G from edl_colsum_bf16_groups
int edl_colsum_bf16_partial(const void* x, int M, int N, float* partial, int G, hipStream_t s) {
  if (N % 8 || G <= 0) return (int)hipErrorInvalidValue;
  int rl = 1;   // row lanes per block: fill the 256 threads when N / 8 < 256
  while (rl < 8 && (N / 8) * rl * 2 <= 256) rl *= 2;
  const dim3 grid((unsigned)((N / 8 + 256 / rl - 1) / (256 / rl)), (unsigned)G);
  switch (rl) {
    case 8: colsum_bf16_partial_kernel<8><<<grid, 256, 0, s>>>((const bf16_t*)x, M, N, partial, G); break;
    case 4: colsum_bf16_partial_kernel<4><<<grid, 256, 0, s>>>((const bf16_t*)x, M, N, partial, G); break;
    case 2: colsum_bf16_partial_kernel<2><<<grid, 256, 0, s>>>((const bf16_t*)x, M, N, partial, G); break;
    default: colsum_bf16_partial_kernel<1><<<grid, 256, 0, s>>>((const bf16_t*)x, M, N, partial, G); break;
  }
  EDL_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
