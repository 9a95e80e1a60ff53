"""Which SDPA flash backends this torch build has (AOTriton / CK) and their times."""
import json
import torch
import torch.nn.functional as F

dev = torch.device("cuda", 0)
out = {"torch": torch.__version__}
try:
    out["preferred"] = str(torch.backends.cuda.preferred_rocm_fa_library())
except Exception as e:
    out["preferred_err"] = repr(e)
q = torch.randn(1, 32, 8192, 128, device=dev, dtype=torch.bfloat16, requires_grad=True)
k = torch.randn(1, 8, 8192, 128, device=dev, dtype=torch.bfloat16, requires_grad=True)
v = torch.randn(1, 8, 8192, 128, device=dev, dtype=torch.bfloat16, requires_grad=True)
do = torch.randn(1, 32, 8192, 128, device=dev, dtype=torch.bfloat16)
for lib in ("aotriton", "ck"):
    try:
        torch.backends.cuda.preferred_rocm_fa_library(lib)
        for _ in range(2):
            F.scaled_dot_product_attention(q, k, v, is_causal=True, enable_gqa=True).backward(do)
        torch.cuda.synchronize()
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        e[0].record()
        for _ in range(5):
            F.scaled_dot_product_attention(q, k, v, is_causal=True, enable_gqa=True)
        e[1].record()
        for _ in range(5):
            F.scaled_dot_product_attention(q, k, v, is_causal=True, enable_gqa=True).backward(do)
        e[2].record()
        torch.cuda.synchronize()
        f = e[0].elapsed_time(e[1]) / 5
        out[lib] = {"fwd_ms": round(f, 3), "bwd_ms": round(e[1].elapsed_time(e[2]) / 5 - f, 3)}
    except Exception as ex:
        out[lib] = repr(ex)[:300]
print(json.dumps(out))
