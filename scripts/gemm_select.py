"""Vet TunableOp GEMM selections one call form at a time and keep only clear wins.

Every GEMM of the Llama-3-8B train step, issued exactly as easydl_amd/ops/fused.py
issues it (M = tokens per micro-batch):

  <lin>.fwd    F.linear(x [M,K], w [N,K])                 lin = qkv, o, lm_head, gate_up, down
  <lin>.dgrad  mm(dy [M,N], wt.t())   wt = W^T [K,N] copy (fused._wt_of)
  <lin>.wgrad  mm(dyT [N,M], xT.t())  transposed activations (NT weight-gradient form)

For each: time with the library heuristic, run a TunableOp search of that one
call, time again.  A selection goes into --out only if it is a hipBLASLt
solution and beats the heuristic by --min-gain in this script's own timing
(round 1 showed TunableOp's isolated wins do not all survive in the step).

    python scripts/gemm_select.py --out easydl_amd/tuned/tunableop_gfx950_select.csv
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=15):
    for _ in range(4):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def forms(M, D=4096, F=14336, Q=6144, V=128256):
    """(name, K, N): y[M,N] = x[M,K] W^T."""
    return [("qkv", D, Q), ("o", D, D), ("gate_up", D, 2 * F), ("down", F, D), ("lm_head", D, V)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=16384)
    ap.add_argument("--min-gain", type=float, default=0.04)
    ap.add_argument("--out", default="")
    ap.add_argument("--only", default="", help="comma list of form names (e.g. down.wgrad)")
    a = ap.parse_args()
    import torch.cuda.tunable as tun
    dev = torch.device("cuda", 0)
    M = a.tokens
    tun.enable(True)
    tun.tuning_enable(False)
    tun.set_max_tuning_duration(60)
    tun.set_max_tuning_iterations(15)
    tun.set_filename(os.path.join("gpurun_out" if os.path.isdir("gpurun_out") else "/tmp", "gemm_select_all_%d.csv"))
    keep = []
    only = set(filter(None, a.only.split(",")))
    for name, K, N in forms(M):
        g = torch.Generator(device=dev).manual_seed(K + N)
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16, generator=g)
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16, generator=g) * 0.02
        dy = torch.randn(M, N, device=dev, dtype=torch.bfloat16, generator=g)
        wt = w.t().contiguous()
        xT, dyT = x.t().contiguous(), dy.t().contiguous()
        dw = torch.empty(N, K, device=dev, dtype=torch.bfloat16)
        ops = {"fwd": lambda: torch.nn.functional.linear(x, w),
               "dgrad": lambda: torch.mm(dy, wt.t()),
               "wgrad": lambda: torch.mm(dyT, xT.t(), out=dw)}
        flops = 2.0 * M * K * N
        for op, fn in ops.items():
            key = f"{name}.{op}"
            if only and key not in only:
                continue
            t0 = timeit(fn)
            before = {tuple(map(str, r[:2])) for r in tun.get_results()}
            tun.tuning_enable(True)
            fn()
            torch.cuda.synchronize()
            tun.tuning_enable(False)
            new = [r for r in tun.get_results() if tuple(map(str, r[:2])) not in before]
            t1 = timeit(fn)
            sol = str(new[0][2]) if new else "?"
            gain = t0 / t1 - 1
            rec = {"form": key, "M": M, "K": K, "N": N, "default_ms": round(t0 * 1e3, 3),
                   "tuned_ms": round(t1 * 1e3, 3), "default_tf": round(flops / t0 / 1e12, 1),
                   "tuned_tf": round(flops / t1 / 1e12, 1), "gain": round(gain, 4), "solution": sol,
                   "kept": bool(new and sol.startswith("Gemm_Hipblaslt") and gain >= a.min_gain)}
            print(json.dumps(rec), flush=True)
            if rec["kept"]:
                keep.append([str(v) for v in new[0]])
        del x, w, dy, wt, xT, dyT, dw, ops
        torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "w") as f:
            vals = tun.get_validators()
            for v in (vals.items() if isinstance(vals, dict) else vals):
                f.write("Validator," + ",".join(map(str, v)) + "\n")
            for r in keep:
                f.write(",".join(r) + "\n")
        print(json.dumps({"written": a.out, "entries": len(keep)}), flush=True)


if __name__ == "__main__":
    main()
