"""Weight-gradient call forms for the BERT-large / Llama-3-8B linear layers (M = 16384
tokens): TN  dW = dY^T X  (one hipBLASLt call on the row-major activations) vs
NT  dW = (dY^T)(X^T)^T  (two LDS-free HIP transposes + the NT GEMM, the framework's
default when the input width is <= 8192).  Times in us, min over 5 x 20 launches."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from easydl_amd.ops.fused import _transposed  # noqa: E402


def bench(fn, it=20):
    best = 1e9
    for _ in range(5):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(it):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / it * 1e3)
    return round(best, 1)


def main():
    M = 16384
    shapes = [("bert_o", 1024, 1024), ("bert_qkv", 3072, 1024), ("bert_fc1", 4096, 1024), ("bert_fc2", 1024, 4096),
              ("llama_o", 4096, 4096), ("llama_qkv", 6144, 4096)]
    for name, N, K in shapes:
        dy = torch.randn(M, N, device="cuda").bfloat16()
        x = torch.randn(M, K, device="cuda").bfloat16()
        out = torch.empty(N, K, device="cuda").bfloat16()
        tn = bench(lambda: torch.mm(dy.t(), x, out=out))

        def nt():
            torch.mm(_transposed(dy), _transposed(x).t(), out=out)
        dyT, xT = _transposed(dy), _transposed(x)
        nt_gemm = bench(lambda: torch.mm(dyT, xT.t(), out=out))
        print(json.dumps({"shape": name, "N": N, "K": K, "TN_us": tn, "NT_with_transposes_us": bench(nt),
                          "NT_gemm_only_us": nt_gemm}), flush=True)


if __name__ == "__main__":
    main()
