"""Weight-gradient GEMM per shape: TN kernel (csrc/kernels/gemm_tn.hip, row-major dY and X)
vs hipBLASLt's NT form on transposed copies (+ the two transposes it needs) and its TN form.
One JSON line per shape (min over reps of cuda-event time)."""
import json
import sys

import torch

from easydl_amd.ops import fused

SHAPES = {  # name: (M, N_out, J_in)
    "bert_qkv": (16384, 3072, 1024), "bert_o": (16384, 1024, 1024), "bert_fc1": (16384, 4096, 1024),
    "bert_fc2": (16384, 1024, 4096), "llama_qkv": (16384, 6144, 4096), "llama_o": (16384, 4096, 4096),
    "llama_gu": (16384, 28672, 4096), "llama_down": (16384, 4096, 14336),
}


def timed(fn, reps=20):
    best = 1e9
    for _ in range(3):
        fn()
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b))
    return best


def main():
    names = sys.argv[1:] or list(SHAPES)
    for name in names:
        M, N, J = SHAPES[name]
        dy = torch.randn(M, N, device="cuda").bfloat16()
        x = torch.randn(M, J, device="cuda").bfloat16()
        out = torch.empty(N, J, device="cuda", dtype=torch.bfloat16)
        ref = torch.mm(dy.t(), x)
        fused.gemm_tn(dy, x, out=out)
        err = ((out.float() - ref.float()).abs().max() / ref.float().abs().max()).item()
        t_tn = timed(lambda: fused.gemm_tn(dy, x, out=out))
        t_tn_acc = timed(lambda: fused.gemm_tn(dy, x, out=out, accumulate=True))
        dyT, xT = fused._transposed(dy), fused._transposed(x)
        t_nt = timed(lambda: torch.mm(dyT, xT.t(), out=out))
        t_tr = timed(lambda: (fused._transposed(dy), fused._transposed(x)))
        t_blas_tn = timed(lambda: torch.mm(dy.t(), x, out=out))
        fl = 2.0 * M * N * J
        print(json.dumps({"shape": name, "M": M, "N": N, "J": J, "rel_err": round(err, 5),
                          "tn_ms": round(t_tn, 4), "tn_acc_ms": round(t_tn_acc, 4), "tn_pf": round(fl / t_tn / 1e12, 3),
                          "nt_ms": round(t_nt, 4), "transposes_ms": round(t_tr, 4),
                          "nt_plus_transposes_ms": round(t_nt + t_tr, 4), "hipblaslt_tn_ms": round(t_blas_tn, 4)}),
              flush=True)


if __name__ == "__main__":
    main()
