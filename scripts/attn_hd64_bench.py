"""Head-dim-64 attention at the BERT-large shape (B 32, S 512, H 16, no mask): our HIP
kernels vs PyTorch SDPA (AOTriton), fwd and fwd+bwd, q/k/v as the strided views of the
fused QKV projection that the model passes.  One JSON line per backend."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from easydl_amd.ops.attention import flash_attention  # noqa: E402


def main():
    B, S, H, D = 32, 512, 16, 64
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = torch.randn(B, S, 3, H, D, device="cuda", generator=g).to(torch.bfloat16)
    do = torch.randn(B, H, S, D, device="cuda", generator=g).to(torch.bfloat16)
    fns = {"hip": lambda q, k, v: flash_attention(q, k, v, causal=False),
           "sdpa": lambda q, k, v: F.scaled_dot_product_attention(q, k, v)}
    outs = {}
    for name, fn in fns.items():
        x = qkv.clone().requires_grad_()
        q, k, v = (t.transpose(1, 2) for t in x.unbind(2))

        def step():
            x.grad = None
            o = fn(q, k, v)
            o.backward(do)
            return o

        o = step()
        outs[name] = (o.detach().float(), x.grad.float())
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        e[0].record()
        for _ in range(20):
            fn(q, k, v)
        e[1].record()
        for _ in range(20):
            step()
        e[2].record()
        torch.cuda.synchronize()
        f, fb = e[0].elapsed_time(e[1]) / 20, e[1].elapsed_time(e[2]) / 20
        fl = 4 * B * H * S * S * D
        print(json.dumps({"backend": name, "fwd_ms": round(f, 4), "fwdbwd_ms": round(fb, 4),
                          "fwd_tflops": round(fl / f / 1e9), "bwd_tflops": round(2.5 * fl / (fb - f) / 1e9)}),
              flush=True)
    d = [((a - b).abs().max() / b.abs().max()).item() for a, b in zip(outs["hip"], outs["sdpa"])]
    print(json.dumps({"hip_vs_sdpa_max_rel_diff": {"o": round(d[0], 5), "dqkv": round(d[1], 5)}}), flush=True)


if __name__ == "__main__":
    main()
