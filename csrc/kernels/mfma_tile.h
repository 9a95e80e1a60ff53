// MFMA tile helpers shared by the hand-written matrix kernels (gemm_tn.hip; the same
// idioms as attention.hip): 256-B-row swizzled LDS tiles that are conflict-free for
// both ds_read_b128 row reads and ds_read_b64_tr_b16 transposed reads
// (cdna_hip_programming.md §5.5 T10 (b)), filled by LDS-DMA (buffer_load ... lds).
#pragma once
#include "common.h"

namespace edl_tile {

using edl::bf16_t;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef short i16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void lds_void;
typedef __amdgpu_buffer_rsrc_t rsrc_t;

// byte offset of 16-B chunk c of row r in a [rows][256 B] LDS tile (XOR swizzle)
__device__ __forceinline__ int swz(int r, int c) { return (r << 8) + ((c ^ (((r & 3) << 2) | ((r >> 2) & 3))) << 4); }
__device__ __forceinline__ int swz_x(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }

__device__ __forceinline__ f32x16 mfma(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// row (within a 32-row block) of accumulator register i for lane half h
__device__ __forceinline__ int acc_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

__device__ __forceinline__ rsrc_t make_rsrc(const void* base, uint32_t nbytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)nbytes, 0x00020000);
}

// 16 B per lane global -> LDS (one wave-instruction = 1 KiB at lds + 16*lane); reads past the
// descriptor's range return zeros.  Device pass only (see attention.hip).
__device__ __forceinline__ void buffer_load_lds16(rsrc_t rs, void* lds, uint32_t voff, uint32_t soff) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)lds, 16, voff, soff, 0, 0);
#endif
}

// LDS-DMA plan for ROWS x 256 B of a row-major matrix (row stride `stride` elements) into
// a swizzled tile: NWAVES waves, each issuing ROWS/4/NWAVES 1-KiB pieces of 4 rows.
template <int ROWS, int NWAVES>
struct DmaPlan {
  static constexpr int PER_WAVE = ROWS / 4 / NWAVES;
  uint32_t voff[PER_WAVE];
  __device__ __forceinline__ DmaPlan(int64_t stride, int w, int lane) {
#pragma unroll
    for (int i = 0; i < PER_WAVE; ++i) {
      const int r = 4 * (w * PER_WAVE + i) + lane / 16;
      const int c = (lane % 16) ^ swz_x(r);
      voff[i] = (uint32_t)((r * stride + c * 8) * 2);
    }
  }
  __device__ __forceinline__ void issue(char* tile, rsrc_t rs, int w) const {
#pragma unroll
    for (int i = 0; i < PER_WAVE; ++i) buffer_load_lds16(rs, tile + (w * PER_WAVE + i) * 1024, voff[i], 0);
  }
};

}  // namespace edl_tile
