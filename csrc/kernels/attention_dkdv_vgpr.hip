// dK/dV attention backward (attn_bwd_dkdv64_kernel, causal, head dim 128) compiled with
// -mllvm --amdgpu-mfma-vgpr-form (easydl_amd/_build.py): MFMA results live in VGPRs, so
// the builtin-MFMA form of the slice (BI = true) needs no inline asm — the compiler sees
// every MFMA, inserts the MFMA -> VALU hazard waits itself and may schedule LDS reads
// and the softmax / dS arithmetic between MFMAs (an inline-asm MFMA is a scheduling
// barrier for both).  Selected by EDL_ATTN_DKDV_MFMA=builtin; =asmvgpr runs the inline-asm
// form under the same flag.  Own translation unit: the flag crashes LLVM 22 on the
// non-causal inline-asm instantiation in attention.hip.
#define EDL_ATTN_VGPR_TU 1
#include "attention.hip"

extern "C" int edl_attn_dkdv64_vgpr(const bf16_t* q, const bf16_t* k, const bf16_t* v, const bf16_t* dout,
                                    const float* lse, const float* delta, void* dk, void* dv, float* ws, unsigned gx,
                                    unsigned gy, unsigned gz, int S, int H, int KV, int gsplit, float sl2, float scale,
                                    int64_t dkvs, int variant, hipStream_t s) {
  const dim3 grid(gx, gy, gz);
  if (variant == 1)
    attn_bwd_dkdv64_kernel<true, 128, true><<<grid, 256, 0, s>>>(q, k, v, dout, lse, delta, (bf16_t*)dk,
                                                                 (bf16_t*)dv, ws, S, H, KV, gsplit, sl2, scale, dkvs);
  else
    attn_bwd_dkdv64_kernel<true, 128, false><<<grid, 256, 0, s>>>(q, k, v, dout, lse, delta, (bf16_t*)dk,
                                                                  (bf16_t*)dv, ws, S, H, KV, gsplit, sl2, scale, dkvs);
  EDL_LAUNCH_CHECK();
  return 0;
}
