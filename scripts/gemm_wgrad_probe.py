"""Down-projection weight gradient of the Llama-3-8B MLP (dW_down [4096, 14336]
= dY^T [4096, M] @ h [M, 14336], M = 16384): the one GEMM of the step that
hipBLASLt's heuristic runs at ~1.1 PF/s (profiles/r02_bench_kernel_stats_mid.csv,
grid 62208).  Times the call as the MLP backward issues it and the
alternatives, one JSON line each:

  current      mm(dyT, hT.t(), out=dw)             (TN, M'=14336 N'=4096)
  current_acc  dw.addmm_(dyT, hT.t())              (second micro-batch)
  swapped      mm(hT, dy, out=dwT)                 (dW^T; + transpose to dW)
  transpose    the [14336, 4096] -> [4096, 14336] transpose alone
  hipblas/ck   current, with rocBLAS / composable_kernel as the preferred library
  tuned        current after a TunableOp search of this one shape

    python scripts/gemm_wgrad_probe.py [--tokens 16384] [--csv out.csv]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=20):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=16384)
    ap.add_argument("--dim", type=int, default=4096)
    ap.add_argument("--ffn", type=int, default=14336)
    ap.add_argument("--csv", default="")
    a = ap.parse_args()
    from easydl_amd import _native
    dev = torch.device("cuda", 0)
    M, D, F = a.tokens, a.dim, a.ffn
    g = torch.Generator(device=dev).manual_seed(0)
    dy = torch.randn(M, D, device=dev, dtype=torch.bfloat16, generator=g)
    hT = torch.randn(F, M, device=dev, dtype=torch.bfloat16, generator=g)
    dyT = dy.t().contiguous()
    dw = torch.empty(D, F, device=dev, dtype=torch.bfloat16)
    dwT = torch.empty(F, D, device=dev, dtype=torch.bfloat16)
    flops = 2.0 * M * D * F
    k = _native.kernels()

    def tr():
        k.check("edl_transpose_bf16", dwT.data_ptr(), dw.data_ptr(), F, D, _native.stream_of(dw))

    ops = {"current": lambda: torch.mm(dyT, hT.t(), out=dw),
           "current_acc": lambda: dw.addmm_(dyT, hT.t()),
           "swapped": lambda: torch.mm(hT, dy, out=dwT),
           "transpose": tr}
    ref = torch.mm(dyT, hT.t()).float()
    for name, fn in ops.items():
        t = timeit(fn)
        print(json.dumps({"op": name, "ms": round(t * 1e3, 3), "tflops": round(flops / t / 1e12, 1)}), flush=True)
    torch.mm(hT, dy, out=dwT)
    tr()
    err = ((dw.float() - ref).abs().max() / ref.abs().max()).item()
    print(json.dumps({"check": "swapped+transpose vs current", "rel_err": err}), flush=True)

    for lib in ("hipblas", "ck"):      # hipblas = rocBLAS on ROCm
        try:
            torch.backends.cuda.preferred_blas_library(lib)
            for name in ("current", "current_acc"):
                t = timeit(ops[name])
                print(json.dumps({"op": f"{lib}_{name}", "ms": round(t * 1e3, 3),
                                  "tflops": round(flops / t / 1e12, 1)}), flush=True)
        except RuntimeError as e:
            print(json.dumps({"op": lib, "error": str(e)[:200]}), flush=True)
    torch.backends.cuda.preferred_blas_library("hipblaslt")

    import torch.cuda.tunable as tun
    tun.enable(True)
    tun.tuning_enable(True)
    tun.set_max_tuning_duration(100)
    tun.set_max_tuning_iterations(20)
    if a.csv:
        tun.set_filename(a.csv)
    for name in ("current", "current_acc"):
        ops[name]()
        torch.cuda.synchronize()
    tun.tuning_enable(False)
    for name in ("current", "current_acc"):
        t = timeit(ops[name])
        print(json.dumps({"op": "tuned_" + name, "ms": round(t * 1e3, 3), "tflops": round(flops / t / 1e12, 1)}),
              flush=True)
    for r in tun.get_results():
        print(json.dumps({"tunableop": [str(x) for x in r]}), flush=True)
    if a.csv:
        tun.write_file()


if __name__ == "__main__":
    main()
