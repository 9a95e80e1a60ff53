"""A/B of attention kernel variants selected by an environment variable, interleaved in
one process at the Llama-3-8B micro-batch shape (B 2, S 8192, H 32, KV 8, causal):
max |difference| between the variants' outputs and gradients, then min-of-5 timings.

    python scripts/attn_variant_ab.py EDL_ATTN_FWD 0 16
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from easydl_amd.ops.attention import flash_attention  # noqa: E402


def mk(B, S, H, KV):
    g = torch.Generator(device="cuda").manual_seed(0)
    return [torch.randn(B, S, n, 128, device="cuda", generator=g).to(torch.bfloat16).transpose(1, 2)
            .requires_grad_() for n in (H, KV, KV)]


def run(q, k, v, do):
    for t in (q, k, v):
        t.grad = None
    o = flash_attention(q, k, v)
    o.backward(do)
    return o.detach(), q.grad, k.grad, v.grad


def main():
    var, vals = sys.argv[1], sys.argv[2:]
    B, S, H, KV = 2, 8192, 32, 8
    q, k, v = mk(B, S, H, KV)
    do = torch.randn(B, H, S, 128, device="cuda").to(torch.bfloat16)
    outs = {}
    for m in vals:
        os.environ[var] = m
        outs[m] = [t.clone() for t in run(q, k, v, do)]
    for m in vals[1:]:
        diff = {n: round(((a.float() - b.float()).abs().max() / b.float().abs().max()).item(), 5)
                for n, a, b in zip(("o", "dq", "dk", "dv"), outs[m], outs[vals[0]])}
        print(json.dumps({"variant": m, "vs": vals[0], "max_rel_diff": diff}), flush=True)
    flops_f = 4 * B * H * S * S * 128 / 2
    res = {m: {"fwd": [], "fwdbwd": []} for m in vals}
    for _ in range(2):
        for m in vals:
            os.environ[var] = m
            run(q, k, v, do)
    torch.cuda.synchronize()
    for _ in range(5):
        for m in vals:
            os.environ[var] = m
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            e[0].record()
            for _ in range(5):
                flash_attention(q, k, v)
            e[1].record()
            for _ in range(5):
                run(q, k, v, do)
            e[2].record()
            torch.cuda.synchronize()
            res[m]["fwd"].append(e[0].elapsed_time(e[1]) / 5)
            res[m]["fwdbwd"].append(e[1].elapsed_time(e[2]) / 5)
    out = {m: {k2: round(min(v2), 4) for k2, v2 in r.items()} for m, r in res.items()}
    for m in out:
        out[m]["fwd_tflops"] = round(flops_f / out[m]["fwd"] / 1e9)
        out[m]["bwd_ms"] = round(out[m]["fwdbwd"] - out[m]["fwd"], 4)
    print(json.dumps({"var": var, "ms_min_B2_S8192_H32_KV8": out}), flush=True)
    # sustained: >= 2 s of back-to-back launches first, so the clock the chip holds under
    # load (MI355X_MICROARCH.md 'DVFS give-back') is what gets timed
    sus = {m: [] for m in vals}
    for _ in range(3):
        for m in vals:
            os.environ[var] = m
            for _ in range(400):
                run(q, k, v, do)
            torch.cuda.synchronize()
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            e[0].record()
            for _ in range(40):
                flash_attention(q, k, v)
            e[1].record()
            for _ in range(20):
                run(q, k, v, do)
            e[2].record()
            torch.cuda.synchronize()
            sus[m].append((e[0].elapsed_time(e[1]) / 40, e[1].elapsed_time(e[2]) / 20))
    print(json.dumps({"var": var, "sustained_ms": {m: {"fwd": round(min(x[0] for x in r), 4),
                                                       "fwdbwd": round(min(x[1] for x in r), 4)}
                                                   for m, r in sus.items()}}), flush=True)


if __name__ == "__main__":
    main()
