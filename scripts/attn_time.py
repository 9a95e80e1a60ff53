"""Flash-attention timings for whichever kernel library EDL_LIBDIR selects: min of 10
cuda-event timings of the forward and of forward + backward.  One JSON line.  Default shape:
the Llama-3-8B micro-batch (B 2, S 8192, H 32, KV 8, causal, head dim 128); `bert`: the
BERT-large batch (B 32, S 512, H 16, bidirectional, head dim 64)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from easydl_amd.ops.attention import flash_attention  # noqa: E402


def main():
    bert = len(sys.argv) > 1 and sys.argv[1] == "bert"
    B, S, H, KV, D, causal = (32, 512, 16, 16, 64, False) if bert else (2, 8192, 32, 8, 128, True)
    g = torch.Generator(device="cuda").manual_seed(0)
    q, k, v = [torch.randn(B, S, n, D, device="cuda", generator=g).bfloat16().transpose(1, 2).requires_grad_()
               for n in (H, KV, KV)]
    do = torch.randn(B, S, H, D, device="cuda", generator=g).bfloat16().transpose(1, 2)

    def fwd():
        with torch.no_grad():
            flash_attention(q, k, v, causal=causal)

    def fwdbwd():
        flash_attention(q, k, v, causal=causal).backward(do)

    out = {"lib": os.environ.get("EDL_LIBDIR", "default"), "shape": "bert" if bert else "llama",
           "short": os.environ.get("EDL_ATTN_SHORT", "1")}
    for name, fn in (("fwd_ms", fwd), ("fwd_bwd_ms", fwdbwd)):
        for _ in range(3):
            fn()
        best = 1e9
        for _ in range(10):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            b.synchronize()
            best = min(best, a.elapsed_time(b))
        out[name] = round(best, 4)
    out["bwd_ms"] = round(out["fwd_bwd_ms"] - out["fwd_ms"], 4)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
