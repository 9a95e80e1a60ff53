"""Per-kernel timing of the flash-attention kernels at the Llama-3-8B shape (and SDPA for reference)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from easydl_amd.ops.attention import flash_attention  # noqa: E402


def run(impl, B=1, S=8192, H=32, KV=8, iters=5):
    os.environ["EDL_ATTN"] = impl
    dev = torch.device("cuda", 0)
    q = torch.randn(B, S, H, 128, device=dev, dtype=torch.bfloat16).transpose(1, 2).requires_grad_()
    k = torch.randn(B, S, KV, 128, device=dev, dtype=torch.bfloat16).transpose(1, 2).requires_grad_()
    v = torch.randn(B, S, KV, 128, device=dev, dtype=torch.bfloat16).transpose(1, 2).requires_grad_()
    if impl == "sdpa":
        q, k, v = (t.detach().transpose(1, 2).contiguous().transpose(1, 2).requires_grad_() for t in (q, k, v))
    o = flash_attention(q, k, v)
    do = torch.randn_like(o)
    for _ in range(2):
        flash_attention(q, k, v).backward(do)
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    e[0].record()
    for _ in range(iters):
        flash_attention(q, k, v)
    e[1].record()
    for _ in range(iters):
        flash_attention(q, k, v).backward(do)
    e[2].record()
    torch.cuda.synchronize()
    flops = 4 * B * H * S * S * 128 / 2
    f = e[0].elapsed_time(e[1]) / iters
    fb = e[1].elapsed_time(e[2]) / iters
    return {"impl": impl, "fwd_ms": round(f, 3), "fwd_tf": round(flops / f / 1e9), "bwd_ms": round(fb - f, 3),
            "bwd_tf": round(2.5 * flops / (fb - f) / 1e9), "fwdbwd_tf": round(3.5 * flops / fb / 1e9)}


if __name__ == "__main__":
    out = [run("hip"), run("sdpa")]
    print(json.dumps(out))
