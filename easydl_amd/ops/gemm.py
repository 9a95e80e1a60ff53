"""Hand-written bf16 NT GEMM for gfx950 (csrc/kernels/gemm_nt.hip):
``C (+)= A @ B^T`` with A [M, K] and B [N, K] both K-contiguous -- the form every large GEMM
of the Llama step takes in this framework's layouts (forward X W^T, input gradient from the
cached W^T, weight gradient from the transposed activations).

``gemm_nt`` runs the kernel when the shape qualifies (M, N multiples of 256, K of 64,
16-byte aligned row strides) and raises otherwise; ``supported`` tells the caller.

Measured (profiles/r05_gemm_nt.md): 1.31-1.34 PF/s on the big Llama-3-8B shapes, 0.80-0.88x of
hipBLASLt's selected solution -- bound by the LDS-DMA load path (~45 GB/s per CU), not by the
MFMA/LDS inner loop (1.63-1.74 PF/s without the loads).  So the training step does not route
any GEMM here; hipBLASLt serves them all.
"""
from __future__ import annotations

import torch

from easydl_amd import _native


def supported(a: torch.Tensor, b: torch.Tensor) -> bool:
    if not (a.is_cuda and b.is_cuda and a.dtype == b.dtype == torch.bfloat16 and a.dim() == 2 and b.dim() == 2):
        return False
    M, K = a.shape
    N, K2 = b.shape
    return (K == K2 and M % 256 == 0 and N % 256 == 0 and K % 64 == 0 and a.stride(1) == 1 and b.stride(1) == 1
            and a.stride(0) % 8 == 0 and b.stride(0) % 8 == 0 and a.data_ptr() % 16 == 0 and b.data_ptr() % 16 == 0)


def gemm_nt(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor | None = None, accumulate: bool = False,
            group_m: int = 8) -> torch.Tensor:
    """``out = a @ b.T`` (or ``out += a @ b.T``), bf16 in/out, fp32 accumulation."""
    if not supported(a, b):
        raise ValueError(f"gemm_nt: unsupported operands {tuple(a.shape)} {a.dtype} x {tuple(b.shape)} {b.dtype}")
    M, K = a.shape
    N = b.shape[0]
    if out is None:
        if accumulate:
            raise ValueError("gemm_nt: accumulate needs out")
        out = torch.empty(M, N, dtype=torch.bfloat16, device=a.device)
    if out.shape != (M, N) or out.dtype != torch.bfloat16 or out.stride(1) != 1 or out.stride(0) % 8 or \
            out.data_ptr() % 16:
        raise ValueError("gemm_nt: out must be a [M, N] bf16 row-major matrix with 16-byte aligned rows")
    _native.kernels().check("edl_gemm_nt", a.data_ptr(), b.data_ptr(), out.data_ptr(), M, N, K, a.stride(0),
                            b.stride(0), out.stride(0), int(accumulate), int(group_m), _native.stream_of(a))
    return out
