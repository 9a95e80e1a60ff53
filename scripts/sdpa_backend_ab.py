"""Time PyTorch SDPA fwd+bwd under each ROCm flash-attention library (AOTriton, CK)
at the BERT-large shape (B 32, S 512, H 16, hd 64, no mask), q/k/v as the strided
views the model passes.  One JSON line per library."""
import json
import sys

import torch
import torch.nn.functional as F


def main():
    B, S, H, D = 32, 512, 16, 64
    libs = sys.argv[1:] or ["aotriton", "ck"]
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = torch.randn(B, S, 3, H, D, device="cuda", generator=g).to(torch.bfloat16)
    do = torch.randn(B, H, S, D, device="cuda", generator=g).to(torch.bfloat16)
    ref = None
    for lib in libs:
        try:
            torch.backends.cuda.preferred_rocm_fa_library(lib)
        except Exception as e:
            print(json.dumps({"lib": lib, "error": str(e)[:200]}), flush=True)
            continue
        x = qkv.clone().requires_grad_()
        q, k, v = (t.transpose(1, 2) for t in x.unbind(2))

        def step():
            x.grad = None
            o = F.scaled_dot_product_attention(q, k, v)
            o.backward(do)
            return o

        try:
            o = step()
        except Exception as e:
            print(json.dumps({"lib": lib, "error": str(e)[:200]}), flush=True)
            continue
        err = None
        if ref is None:
            ref = (o.detach().float(), x.grad.float())
        else:
            err = [((a.float() - b).abs().max() / b.abs().max()).item() for a, b in ((o, ref[0]), (x.grad, ref[1]))]
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        e[0].record()
        for _ in range(20):
            F.scaled_dot_product_attention(q, k, v)
        e[1].record()
        for _ in range(20):
            step()
        e[2].record()
        torch.cuda.synchronize()
        f = e[0].elapsed_time(e[1]) / 20
        fb = e[1].elapsed_time(e[2]) / 20
        fl = 4 * B * H * S * S * D
        print(json.dumps({"lib": lib, "fwd_ms": round(f, 3), "fwdbwd_ms": round(fb, 3),
                          "fwd_tflops": round(fl / f / 1e9), "bwd_tflops": round(2.5 * fl / (fb - f) / 1e9),
                          "rel_err_vs_first": err}), flush=True)


if __name__ == "__main__":
    main()
