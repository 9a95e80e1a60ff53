"""Hand-written NT GEMM vs hipBLASLt (the trainer's TunableOp selections) on the Llama-3-8B
shapes, interleaved in one process (cdna_hip_programming.md §5.4 rule 24), random data.

    python scripts/gemm_nt_bench.py [--rounds 5] [--group 8]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--group", type=int, default=8)
    ap.add_argument("--tokens", type=int, default=16384)
    ap.add_argument("--only", default="")
    ap.add_argument("--arms", default="", help="kernel arms name:flags:group_m,... (the 8-phase kernel)")
    ap.add_argument("--diag", action="store_true", help="also time the kernel without DMA, the DMA alone, and F.linear")
    a = ap.parse_args()
    from easydl_amd.ops import gemm_tuning
    from easydl_amd.ops.gemm import gemm_nt
    from easydl_amd import _native
    gemm_tuning.apply("select")
    dev = torch.device("cuda", 0)
    T = a.tokens
    # (name, M, N, K): C[M, N] = A[M, K] B[N, K]^T
    shapes = [("qkv.fwd", T, 6144, 4096), ("o.fwd", T, 4096, 4096), ("gate_up.fwd", T, 28672, 4096),
              ("down.fwd", T, 4096, 14336), ("lm_head.fwd", T, 128256, 4096),
              ("qkv.dgrad", T, 4096, 6144), ("gate_up.dgrad", T, 4096, 28672), ("down.dgrad", T, 14336, 4096),
              ("qkv.wgrad", 6144, 4096, T), ("o.wgrad", 4096, 4096, T), ("gate_up.wgrad", 28672, 4096, T),
              ("down.wgrad", 4096, 14336, T)]
    if a.only:
        shapes = [s for s in shapes if s[0] in a.only.split(",")]
    for name, M, N, K in shapes:
        A = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        B = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
        C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        ref = torch.mm(A, B.t())
        gemm_nt(A, B, out=C, group_m=a.group)
        rel = ((C.float() - ref.float()).norm() / ref.float().norm()).item()
        flops = 2.0 * M * N * K
        res = {"edl": [], "hipblaslt": []}
        C8 = torch.empty_like(C)
        arms = {}
        for spec in (a.arms.split(",") if a.arms else []):
            nm, flag, grp = spec.split(":")[:3]
            fn_name = "edl_gemm_nt8"
            arms[nm] = (lambda flag=int(flag), grp=int(grp), fn_name=fn_name: _native.kernels().check(
                fn_name, A.data_ptr(), B.data_ptr(), C8.data_ptr(), M, N, K, K, K, N, flag, grp,
                _native.stream_of(A)))
        rels = {}
        for nm, fn in arms.items():
            C8.zero_()
            fn()
            rels[nm] = round(((C8.float() - ref.float()).norm() / ref.float().norm()).item(), 5)
            res[nm] = []

        def timed(fn):
            fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.iters):
                fn()
            torch.cuda.synchronize()
            return (time.perf_counter() - t0) / a.iters

        k = _native.kernels()

        def diag(mode):
            k.check("edl_gemm_nt_diag", A.data_ptr(), B.data_ptr(), C.data_ptr(), M, N, K, K, K, N, mode, a.group,
                    _native.stream_of(A))
        if a.diag:
            res.update({"diag_no_dma": [], "diag_dma_only": [], "F.linear": []})
        for _ in range(a.rounds):
            res["edl"].append(timed(lambda: gemm_nt(A, B, out=C, group_m=a.group)))
            res["hipblaslt"].append(timed(lambda: torch.mm(A, B.t(), out=C)))
            for nm, fn in arms.items():
                res[nm].append(timed(fn))
            if a.diag:
                res["diag_no_dma"].append(timed(lambda: diag(1)))
                res["diag_dma_only"].append(timed(lambda: diag(2)))
                res["F.linear"].append(timed(lambda: torch.nn.functional.linear(A, B)))

        out = {"shape": name, "M": M, "N": N, "K": K, "rel_err_vs_hipblaslt": round(rel, 5), "group_m": a.group}
        for k, v in res.items():
            best = min(v)
            out[k] = {"ms": round(best * 1e3, 4), "tflops": round(flops / best / 1e12, 1),
                      "median_ms": round(sorted(v)[len(v) // 2] * 1e3, 4)}
        out["speedup"] = round(out["hipblaslt"]["ms"] / out["edl"]["ms"], 3)
        for nm in arms:
            out[nm]["rel_err"] = rels[nm]
            out[nm]["vs_hipblaslt"] = round(out["hipblaslt"]["ms"] / out[nm]["ms"], 3)
        print(json.dumps(out), flush=True)
        del A, B, C, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
