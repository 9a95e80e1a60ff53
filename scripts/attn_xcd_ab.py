"""A/B of the XCD-aware work decode of the attention forward and dQ kernels
(EDL_ATTN_XCD=0/1), interleaved in one process at the Llama-3-8B micro-batch shape.
Both mappings run the same per-workgroup arithmetic, so outputs must be bitwise equal."""
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
    B, S, H, KV = 2, 8192, 32, 8
    q, k, v = mk(B, S, H, KV)
    do = torch.randn(B, H, S, 128, device="cuda").to(torch.bfloat16)
    outs = {}
    for m in ("0", "1"):
        os.environ["EDL_ATTN_XCD"] = m
        outs[m] = [t.clone() for t in run(q, k, v, do)]
    same = all(torch.equal(a, b) for a, b in zip(outs["0"], outs["1"]))
    print(json.dumps({"bitwise_equal": same}), flush=True)
    flops_f = 4 * B * H * S * S * 128 / 2
    res = {m: {"fwd": [], "fwdbwd": []} for m in ("0", "1")}
    for _ in range(2):
        for m in ("0", "1"):
            os.environ["EDL_ATTN_XCD"] = m
            run(q, k, v, do)
    torch.cuda.synchronize()
    for _ in range(5):
        for m in ("0", "1"):
            os.environ["EDL_ATTN_XCD"] = m
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
    print(json.dumps({"ms_min_B2_S8192_H32_KV8": out}), flush=True)


if __name__ == "__main__":
    main()
