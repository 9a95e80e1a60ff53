"""Per-shape GEMM throughput of the Llama-3-8B train step (fwd, dgrad, wgrad)
with the library's default heuristics and, with --tune, PyTorch TunableOp
(hipBLASLt + rocBLAS solution search).  Writes one JSON line per shape.

    python scripts/gemm_bench.py --tokens 16384 [--tune --tune-file easydl_amd/tuned/gemm_gfx950.csv]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def shapes(model: str):
    from easydl_amd.models.llama import get_config
    c = get_config(model)
    hd = c.dim // c.n_heads
    return {"qkv": (c.dim, (c.n_heads + 2 * c.n_kv_heads) * hd), "o": (c.dim, c.dim),
            "gate_up": (c.dim, 2 * c.ffn_dim), "down": (c.ffn_dim, c.dim), "lm_head": (c.dim, c.vocab_size)}


def tr(src, dst):
    from easydl_amd import _native
    _native.kernels().check("edl_transpose_bf16", src.data_ptr(), dst.data_ptr(), src.shape[0], src.shape[1],
                            _native.stream_of(src))


def timeit(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--tokens", type=int, default=16384)
    ap.add_argument("--tune", action="store_true")
    ap.add_argument("--tune-file", default="")
    ap.add_argument("--out", default="")
    ap.add_argument("--layouts", action="store_true", help="also time the W^T [in,out] storage variants")
    ap.add_argument("--blas", default="", help="hipblaslt | rocblas (torch.backends.cuda.preferred_blas_library)")
    ap.add_argument("--select", action="store_true", help="the trainer's GEMM configuration (shipped TunableOp "
                                                               "selections, easydl_amd/ops/gemm_tuning.py)")
    a = ap.parse_args()
    if a.select:
        from easydl_amd.ops import gemm_tuning
        print(json.dumps({"gemm_tuning": gemm_tuning.apply("select")}), flush=True)
    if a.blas:
        torch.backends.cuda.preferred_blas_library(a.blas)
    if a.tune:
        import torch.cuda.tunable as tun
        tun.enable(True)
        tun.tuning_enable(True)
        if a.tune_file:
            tun.set_filename(a.tune_file)
        tun.set_max_tuning_duration(200)
    dev = torch.device("cuda", 0)
    M = a.tokens
    res = []
    total = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}
    for name, (k, n) in shapes(a.model).items():
        x = torch.randn(M, k, device=dev, dtype=torch.bfloat16)
        w = torch.randn(n, k, device=dev, dtype=torch.bfloat16) * 0.02
        dy = torch.randn(M, n, device=dev, dtype=torch.bfloat16)
        dw = torch.empty(n, k, device=dev, dtype=torch.bfloat16)
        flops = 2.0 * M * k * n
        wt = w.t().contiguous()          # alternative storage: W^T [in, out] row-major
        dyT, xT = dy.t().contiguous(), x.t().contiguous()
        dwt = torch.empty(k, n, device=dev, dtype=torch.bfloat16)
        ops = {"fwd": lambda: torch.nn.functional.linear(x, w),
               "dgrad": lambda: torch.mm(dy, w),
               "wgrad": lambda: torch.mm(dy.t(), x, out=dw),
               "wgrad_acc": lambda: dw.addmm_(dy.t(), x)}
        if a.layouts:
            ops.update({"T_fwd": lambda: torch.mm(x, wt),
                        "T_dgrad": lambda: torch.mm(dy, wt.t()),
                        "T_wgrad": lambda: torch.mm(x.t(), dy, out=dwt),
                        # wgrad in NT form from transposed activations (dY^T [N,M], X^T [K,M] contiguous)
                        "NT_wgrad": lambda: torch.mm(dyT, xT.t(), out=dw),
                        "transpose_dy_x": lambda: (tr(dy, dyT), tr(x, xT))})
        for op, fn in ops.items():
            t = timeit(fn)
            r = {"shape": name, "op": op, "M": M, "K": k, "N": n, "ms": round(t * 1e3, 3),
                 "tflops": round(flops / t / 1e12, 1), "tuned": a.tune, "blas": a.blas or "default"}
            if op in total:
                total[op] += t
            res.append(r)
            print(json.dumps(r), flush=True)
        del x, w, dy, dw, wt, dwt, dyT, xT
        torch.cuda.empty_cache()
    print(json.dumps({"total_ms": {k: round(v * 1e3, 2) for k, v in total.items()}}), flush=True)
    if a.tune:
        import torch.cuda.tunable as tun
        tun.write_file()
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
