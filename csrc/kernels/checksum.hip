// Block checksum of device buffers for in-memory snapshot integrity
// (SURVEY.md §2.4 N11, K11).  checksum = sum_i w_i * (2i + 1)  (mod 2^64) over
// the buffer's 32-bit words w_i: integer arithmetic, so the result is
// independent of reduction order (bitwise reproducible), and any single-word
// corruption or word swap changes it.  HBM-bound: 16-B loads, per-block
// partial in registers/LDS, one 64-bit atomic per block.
#include "common.h"

using namespace edl;

namespace {

__global__ __launch_bounds__(256) void checksum_kernel(const uint32_t* __restrict__ w, int64_t nwords,
                                                       unsigned long long* __restrict__ out, uint64_t base_index) {
  __shared__ unsigned long long red[4];
  unsigned long long acc = 0;
  const int64_t n4 = nwords >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const u32x4 v = reinterpret_cast<const u32x4*>(w)[i];
    const uint64_t k = base_index + (uint64_t)i * 4;
#pragma unroll
    for (int j = 0; j < 4; ++j) acc += (unsigned long long)v[j] * (2ull * (k + j) + 1ull);
  }
  if (blockIdx.x == 0 && threadIdx.x < (nwords & 3)) {
    const int64_t j = n4 * 4 + threadIdx.x;
    acc += (unsigned long long)w[j] * (2ull * (base_index + (uint64_t)j) + 1ull);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += red[i];
    atomicAdd(out, t);
  }
}

}  // namespace

extern "C" {

// Adds the checksum of [ptr, ptr+nbytes) (nbytes % 4 == 0, ptr 16-B aligned) to
// *out (caller zeroes it).  base_index offsets the word positions so a buffer
// checksummed in pieces equals the checksum of the whole.
int edl_checksum(const void* ptr, int64_t nbytes, unsigned long long* out, uint64_t base_index, hipStream_t s) {
  if (nbytes % 4) return (int)hipErrorInvalidValue;
  const int64_t nwords = nbytes / 4;
  int64_t blocks = (nwords / 4 + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (blocks > 2048) blocks = 2048;
  checksum_kernel<<<(int)blocks, 256, 0, s>>>((const uint32_t*)ptr, nwords, out, base_index);
  EDL_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
