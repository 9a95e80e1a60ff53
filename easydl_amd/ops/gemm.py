"""Hand-written bf16 NT GEMM for gfx950 (csrc/kernels/gemm_nt.hip; the reference publishes no
kernels -- its training performance claim is /root/reference/README.md:19-23):
``C (+)= A @ B^T`` with A [M, K] and B [N, K] both K-contiguous -- the form every large GEMM
of the Llama step takes in this framework's layouts (forward X W^T, input gradient from the
cached W^T, weight gradient from the transposed activations).

``gemm_nt`` runs the kernel when the shape qualifies (M, N multiples of 256, K of 64,
16-byte aligned row strides) and raises otherwise; ``supported`` tells the caller.

Two kernels.  ``kernel="nt"`` (round 5, profiles/r05_gemm_nt.md): two LDS stages, one
``vmcnt(0)`` + barrier per K-tile, 1.31-1.34 PF/s.  ``kernel="nt8"`` (round 6,
profiles/r06_gemm_nt8.md): the 8-phase ping-pong pipeline with counted ``vmcnt`` and the next
tile's B fragments read ahead, 1.49-1.60 PF/s = 0.93-1.04x hipBLASLt's selected solution.  Both
sit at the same power-limited clock (~1.75 GHz) and MFMA share as hipBLASLt in PMC; the step
routes only the shape where nt8 wins (the gate/up input gradient, ops/fused.py
``EDL_GEMM_NT8_DGRAD``).
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
            group_m: int = 8, kernel: str = "nt") -> torch.Tensor:
    """``out = a @ b.T`` (or ``out += a @ b.T``), bf16 in/out, fp32 accumulation.  ``kernel``:
    "nt" (round 5) or "nt8" (8-phase, K a multiple of 128 for the B read-ahead)."""
    if not supported(a, b) or (kernel == "nt8" and a.shape[1] < 128):
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
    name, flags = ("edl_gemm_nt8", int(accumulate) | 2) if kernel == "nt8" else ("edl_gemm_nt", int(accumulate))
    _native.kernels().check(name, a.data_ptr(), b.data_ptr(), out.data_ptr(), M, N, K, a.stride(0),
                            b.stride(0), out.stride(0), flags, int(group_m), _native.stream_of(a))
    return out
