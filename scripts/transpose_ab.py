"""A/B of the transposed-output kernels (csrc/kernels/fused.hip): the register
8x8-block versions (edl_transpose_bf16, edl_swiglu_{fwd,bwd}_t) against the
LDS-tile versions (*_lds), on the Llama-3-8B train-step shapes (16384 tokens).
Checks the two agree bit for bit, prints one JSON line per (kernel, shape) with
ms and effective HBM TB/s.

    python scripts/transpose_ab.py [--out gpurun_out/transpose_ab.jsonl]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from easydl_amd import _native  # noqa: E402


def timeit(fn, iters=20):
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
    ap.add_argument("--tokens", type=int, default=16384)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    k = _native.kernels()
    dev = torch.device("cuda", 0)
    M = a.tokens
    rows = []
    st = torch.cuda.current_stream().cuda_stream
    for name, C in (("x_dim", 4096), ("qkv", 6144), ("ffn", 14336), ("gate_up", 28672)):
        x = torch.randn(M, C, device=dev, dtype=torch.bfloat16)
        ys = {v: torch.empty(C, M, device=dev, dtype=torch.bfloat16) for v in ("reg", "lds")}
        for v, fn in (("reg", "edl_transpose_bf16"), ("lds", "edl_transpose_bf16_lds")):
            call = lambda fn=fn, y=ys[v]: k.check(fn, x.data_ptr(), y.data_ptr(), M, C, st)  # noqa: E731
            ms = timeit(call) * 1e3
            rows.append({"kernel": "transpose", "variant": v, "shape": [M, C], "ms": round(ms, 4),
                         "tb_s": round(4 * M * C / ms / 1e9, 3)})
        assert torch.equal(ys["reg"], ys["lds"]) and torch.equal(ys["reg"], x.t()), name
        del x, ys
    F = 14336
    gu = torch.randn(M, 2 * F, device=dev, dtype=torch.bfloat16)
    dh = torch.randn(M, F, device=dev, dtype=torch.bfloat16)
    outs = {}
    for v, sfx in (("reg", ""), ("lds", "_lds")):
        h = torch.empty(M, F, device=dev, dtype=torch.bfloat16)
        hT = torch.empty(F, M, device=dev, dtype=torch.bfloat16)
        ms = timeit(lambda: k.check("edl_swiglu_fwd_t" + sfx, gu.data_ptr(), h.data_ptr(), hT.data_ptr(),
                                    M, F, st)) * 1e3
        rows.append({"kernel": "swiglu_fwd_t", "variant": v, "shape": [M, F], "ms": round(ms, 4),
                     "tb_s": round(2 * M * F * 4 / ms / 1e9, 3)})
        dgu, dguT = torch.empty_like(gu), torch.empty(2 * F, M, device=dev, dtype=torch.bfloat16)
        ms = timeit(lambda: k.check("edl_swiglu_bwd_t" + sfx, dh.data_ptr(), gu.data_ptr(), dgu.data_ptr(),
                                    dguT.data_ptr(), M, F, st)) * 1e3
        rows.append({"kernel": "swiglu_bwd_t", "variant": v, "shape": [M, F], "ms": round(ms, 4),
                     "tb_s": round(2 * M * F * 7 / ms / 1e9, 3)})
        outs[v] = (h, hT, dgu, dguT)
    for i in range(4):
        assert torch.equal(outs["reg"][i], outs["lds"][i]), i
    assert torch.equal(outs["reg"][1], outs["reg"][0].t()) and torch.equal(outs["reg"][3], outs["reg"][2].t())
    lines = [json.dumps(r) for r in rows]
    print("\n".join(lines), flush=True)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
