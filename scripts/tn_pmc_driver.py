"""Runs the TN weight-gradient kernels on the Llama gate/up shape (256 x 256 kernel, EDL_WGRAD
default) and the BERT fc1 shape (128 x 256 split kernel) a few times each: a short program for
rocprofv3 --pmc passes."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from easydl_amd.ops import fused  # noqa: E402

for M, N, J in ((16384, 28672, 4096), (16384, 4096, 1024)):
    dy = torch.randn(M, N, device="cuda").bfloat16()
    x = torch.randn(M, J, device="cuda").bfloat16()
    out = torch.empty(N, J, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        fused.gemm_tn(dy, x, out=out)
    torch.cuda.synchronize()
