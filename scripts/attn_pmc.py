"""Run only the hand-written attention kernels a few times (for rocprofv3 --pmc)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["EDL_ATTN"] = "hip"
from easydl_amd.ops.attention import flash_attention  # noqa: E402

dev = torch.device("cuda", 0)
B, S, H, KV = int(os.environ.get("B", 2)), int(os.environ.get("S", 8192)), 32, 8
q = torch.randn(B, S, H, 128, device=dev, dtype=torch.bfloat16).transpose(1, 2).requires_grad_()
k = torch.randn(B, S, KV, 128, device=dev, dtype=torch.bfloat16).transpose(1, 2).requires_grad_()
v = torch.randn(B, S, KV, 128, device=dev, dtype=torch.bfloat16).transpose(1, 2).requires_grad_()
do = torch.randn(B, H, S, 128, device=dev, dtype=torch.bfloat16)
for _ in range(int(os.environ.get("ITERS", 3))):
    flash_attention(q, k, v).backward(do)
torch.cuda.synchronize()
print("ok")
