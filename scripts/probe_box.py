"""Probe the MI355X box: memory, GEMM rates (hipBLASLt via torch), SDPA backends/speed."""
import json
import os
import time
import torch
import torch.nn.functional as F

out = {}
out["torch"] = torch.__version__
out["hip"] = torch.version.hip
p = torch.cuda.get_device_properties(0)
out["dev"] = {"name": p.name, "cus": p.multi_processor_count, "mem_gb": p.total_memory / 2**30,
              "gcn": getattr(p, "gcnArchName", "")}
try:
    out["host_mem_gb"] = os.sysconf("SC_PAGE_SIZE") * os.sysconf("SC_PHYS_PAGES") / 2**30
except Exception:
    pass

def bench(fn, iters=20, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters

dt = torch.bfloat16
gemm = {}
T = 8192
for (m, k, n, name) in [(T, 4096, 6144, "qkv"), (T, 4096, 4096, "o"), (T, 4096, 28672, "gateup"),
                        (T, 14336, 4096, "down"), (T, 4096, 128256, "lmhead"),
                        (4096, T, 14336, "dW_down_like"), (8192, 8192, 8192, "sq8k")]:
    a = torch.randn(m, k, device="cuda", dtype=dt)
    b = torch.randn(k, n, device="cuda", dtype=dt)
    s = bench(lambda: a @ b)
    gemm[name] = {"shape": [m, k, n], "ms": s * 1e3, "tflops": 2 * m * k * n / s / 1e12}
    # transposed-weight layout (nn.Linear style: x @ W^T with W [n,k])
    w = torch.randn(n, k, device="cuda", dtype=dt)
    s2 = bench(lambda: F.linear(a, w))
    gemm[name]["linear_tflops"] = 2 * m * k * n / s2 / 1e12
    del a, b, w
out["gemm"] = gemm

att = {}
B, H, HKV, S, D = 1, 32, 8, 8192, 128
q = torch.randn(B, H, S, D, device="cuda", dtype=dt, requires_grad=True)
k = torch.randn(B, HKV, S, D, device="cuda", dtype=dt, requires_grad=True)
v = torch.randn(B, HKV, S, D, device="cuda", dtype=dt, requires_grad=True)
from torch.nn.attention import sdpa_kernel, SDPBackend
for be in [SDPBackend.FLASH_ATTENTION, SDPBackend.EFFICIENT_ATTENTION, SDPBackend.CUDNN_ATTENTION, SDPBackend.MATH]:
    if be == SDPBackend.MATH:
        continue
    try:
        with sdpa_kernel([be]):
            f = lambda: F.scaled_dot_product_attention(q, k, v, is_causal=True, enable_gqa=True)
            s = bench(f, iters=10)
            o = f()
            g = torch.randn_like(o)
            def fb():
                o = F.scaled_dot_product_attention(q, k, v, is_causal=True, enable_gqa=True)
                o.backward(g)
            sb = bench(fb, iters=5, warm=2)
        flops = 4 * B * H * S * S * D / 2
        att[str(be)] = {"fwd_ms": s * 1e3, "fwd_tflops": flops / s / 1e12, "fwdbwd_ms": sb * 1e3,
                        "fwdbwd_tflops": 3.5 * flops / sb / 1e12}
    except Exception as e:
        att[str(be)] = {"error": repr(e)[:300]}
out["sdpa"] = att
# HBM copy bandwidth
x = torch.empty(2**30, device="cuda", dtype=torch.float32)
y = torch.empty_like(x)
s = bench(lambda: y.copy_(x), iters=10)
out["copy_TBps"] = 2 * x.numel() * 4 / s / 1e12
del x, y
print(json.dumps(out, indent=1))
os.makedirs("gpurun_out", exist_ok=True)
with open("gpurun_out/probe.json", "w") as f:
    json.dump(out, f, indent=1)
