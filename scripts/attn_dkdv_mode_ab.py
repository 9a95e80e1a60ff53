"""A/B of the dK/dV work order (EDL_ATTN_DKDV_MODE bit 0: whole K/V groups per XCD;
bit 1: descending, head-fastest query sweep) at the Llama-3-8B micro-batch shape.
Numerics vs mode 0 first (summation order differs: tolerance, not bitwise)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from easydl_amd.ops.attention import flash_attention  # noqa: E402

MODES = ["0", "1", "2", "3"]


def main():
    B, S, H, KV = 2, 8192, 32, 8
    g = torch.Generator(device="cuda").manual_seed(0)
    q, k, v = [torch.randn(B, S, n, 128, device="cuda", generator=g).to(torch.bfloat16).transpose(1, 2)
               .requires_grad_() for n in (H, KV, KV)]
    do = torch.randn(B, H, S, 128, device="cuda", generator=g).to(torch.bfloat16)
    o = flash_attention(q, k, v)
    grads = {}
    for m in MODES:
        os.environ["EDL_ATTN_DKDV_MODE"] = m
        k.grad = v.grad = q.grad = None
        o.backward(do, retain_graph=True)
        grads[m] = (k.grad.float().clone(), v.grad.float().clone())
    err = {m: max(((a - b).abs().max() / b.abs().max()).item() for a, b in zip(grads[m], grads["0"]))
           for m in MODES}
    print(json.dumps({"rel_err_vs_mode0": err}), flush=True)
    res = {m: [] for m in MODES}
    for _ in range(2):
        for m in MODES:
            os.environ["EDL_ATTN_DKDV_MODE"] = m
            o.backward(do, retain_graph=True)
    torch.cuda.synchronize()
    for _ in range(5):
        for m in MODES:
            os.environ["EDL_ATTN_DKDV_MODE"] = m
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                o.backward(do, retain_graph=True)
            e1.record()
            torch.cuda.synchronize()
            res[m].append(e0.elapsed_time(e1) / 5)
    print(json.dumps({"bwd_ms_min": {m: round(min(t), 4) for m, t in res.items()},
                      "bwd_ms_med": {m: round(sorted(t)[2], 4) for m, t in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
