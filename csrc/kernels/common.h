// Shared device helpers for the easydl_amd CDNA4 (gfx950) kernel library.
//
// Design notes (MI355X-first, see docs/kernels.md):
//  * 64-lane wavefronts: every reduction is a 64-wide shuffle tree, block
//    sizes are multiples of 64.
//  * All memory-bound kernels move 8-16 B per lane per access
//    (cdna_hip_programming.md Guideline 13); bf16 is handled as raw uint16
//    bit patterns so loads stay vectorised.
//  * No CUDA shims / dual paths: this code targets gfx950 only.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace edl {

typedef uint16_t bf16_t;
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;

__device__ __forceinline__ float bf2f(bf16_t x) { return __uint_as_float(((uint32_t)x) << 16); }
__device__ __forceinline__ float bflo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bfhi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

// fp32 -> bf16, round-to-nearest-even, quiet NaNs preserved.
__device__ __forceinline__ uint32_t f2bf_bits(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return ((u >> 16) | 0x40u) & 0xffffu;
  u += 0x7fffu + ((u >> 16) & 1u);
  return u >> 16;
}
__device__ __forceinline__ bf16_t f2bf(float f) { return (bf16_t)f2bf_bits(f); }
__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
  return f2bf_bits(lo) | (f2bf_bits(hi) << 16);
}

// 8 bf16 packed in 16 bytes <-> 8 floats.
__device__ __forceinline__ void unpack8(const u32x4& v, float (&f)[8]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = bflo(v[i]);
    f[2 * i + 1] = bfhi(v[i]);
  }
}
__device__ __forceinline__ u32x4 pack8(const float (&f)[8]) {
  u32x4 v;
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = pack2(f[2 * i], f[2 * i + 1]);
  return v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, kWave));
  return v;
}

// Block-wide sum; `red` must hold >= blockDim/64 floats. All threads get the result.
__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_sum(v);
  __syncthreads();  // protect `red` reuse across consecutive calls
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }

}  // namespace edl

#define EDL_LAUNCH_CHECK() \
  do {                     \
    hipError_t e__ = hipGetLastError(); \
    if (e__ != hipSuccess) return (int)e__; \
  } while (0)
