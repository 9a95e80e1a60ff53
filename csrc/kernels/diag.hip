// Hardware probes used by scripts (not on any training path).
//
// edl_diag_lds_dma: copy 1 KiB from global memory into LDS at byte offset
// `off` of a 160 KiB workgroup allocation with one LDS-DMA wave instruction
// (buffer_load_dwordx4 ... lds), then read it back with ds_read and store it.
// Answers whether LDS-DMA destinations above 64 KiB land where M0 points.
#include "common.h"

using namespace edl;

namespace {
typedef __attribute__((address_space(3))) void lds_void;

__global__ __launch_bounds__(64) void diag_lds_dma_kernel(const uint32_t* __restrict__ src, uint32_t* __restrict__ out,
                                                          int off) {
  __shared__ __attribute__((aligned(16))) char smem[160 * 1024];
  const int lane = threadIdx.x;
  // poison the whole target window first
  for (int i = lane; i < 256; i += 64) reinterpret_cast<uint32_t*>(smem + off)[i] = 0xDEADBEEFu;
  __syncthreads();
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(src), (short)0, 1024, 0x00020000);
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(smem + off), 16, (uint32_t)lane * 16, 0, 0, 0);
#endif
  __builtin_amdgcn_s_waitcnt(0x0F70);
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i) out[lane * 4 + i] = reinterpret_cast<const uint32_t*>(smem + off)[lane * 4 + i];
  // and what landed at off - 64 KiB (a wrapped 16-bit address would land there)
  if (off >= 65536) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      out[256 + lane * 4 + i] = reinterpret_cast<const uint32_t*>(smem + off - 65536)[lane * 4 + i];
  }
}
}  // namespace

extern "C" int edl_diag_lds_dma(const void* src, void* out, int off, hipStream_t s) {
  if (off < 0 || off + 1024 > 160 * 1024 || (off & 15)) return (int)hipErrorInvalidValue;
  diag_lds_dma_kernel<<<1, 64, 0, s>>>((const uint32_t*)src, (uint32_t*)out, off);
  EDL_LAUNCH_CHECK();
  return 0;
}
