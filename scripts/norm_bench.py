"""RMSNorm / LayerNorm fwd+bwd timing at the Llama-3-8B (16384 x 4096) and BERT-large
(16384 x 1024) micro-batch shapes, fused residual add included.  One JSON line per case."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from easydl_amd.ops import norms  # noqa: E402


def bench(kind, rows, cols, iters=20):
    dev = torch.device("cuda")
    x = torch.randn(rows, cols, device=dev, dtype=torch.bfloat16, requires_grad=True)
    r = torch.randn(rows, cols, device=dev, dtype=torch.bfloat16, requires_grad=True)
    w = torch.ones(cols, device=dev, dtype=torch.bfloat16, requires_grad=True)
    b = torch.zeros(cols, device=dev, dtype=torch.bfloat16, requires_grad=True)
    if kind == "rms":
        fn = lambda: norms.add_rmsnorm(x, r, w, 1e-5)  # noqa: E731
    else:
        fn = lambda: norms.add_layernorm(x, r, w, b, 1e-5)  # noqa: E731
    y, s = fn()
    gy, gs = torch.randn_like(y), torch.randn_like(s)
    for _ in range(3):
        y, s = fn()
        torch.autograd.backward([y, s], [gy, gs])
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    e[0].record()
    for _ in range(iters):
        y, s = fn()
    e[1].record()
    for _ in range(iters):
        y, s = fn()
        torch.autograd.backward([y, s], [gy, gs])
    e[2].record()
    torch.cuda.synchronize()
    f = e[0].elapsed_time(e[1]) / iters
    fb = e[1].elapsed_time(e[2]) / iters - f
    gb = rows * cols * 2 / 1e9
    print(json.dumps({"kind": kind, "rows": rows, "cols": cols, "fwd_us": round(f * 1e3, 1),
                      "bwd_us": round(fb * 1e3, 1), "fwd_TBps": round(4 * gb / f, 2),
                      "bwd_TBps_3read1write": round(4 * gb / fb, 2)}), flush=True)


if __name__ == "__main__":
    bench("rms", 16384, 4096)
    bench("ln", 16384, 1024)
