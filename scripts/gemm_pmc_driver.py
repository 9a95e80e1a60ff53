"""Kernel driver for rocprofv3 PMC passes over the 8-phase NT GEMM and hipBLASLt on one
Llama-3-8B shape (scripts/gpu/pmc.sh DRIVER=scripts/gemm_pmc_driver.py); random operands.

    python scripts/gemm_pmc_driver.py [shape M N K] [flags group_m]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from easydl_amd import _native
    from easydl_amd.ops import gemm_tuning
    gemm_tuning.apply("select")
    M, N, K = (int(x) for x in os.environ.get("GEMM_SHAPE", "16384,28672,4096").split(","))
    flags, grp = (int(x) for x in os.environ.get("GEMM_ARM", "2,8").split(","))
    dev = torch.device("cuda", 0)
    A = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
    B = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
    C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    k = _native.kernels()
    for _ in range(int(os.environ.get("GEMM_ITERS", "20"))):
        k.check("edl_gemm_nt8", A.data_ptr(), B.data_ptr(), C.data_ptr(), M, N, K, K, K, N, flags, grp,
                _native.stream_of(A))
        torch.mm(A, B.t(), out=C)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
