"""Only the flash-attention FORWARD kernels, both variants (for rocprofv3 --pmc):
EDL_ATTN_FWD=0 then 64, B=2 S=8192 H=32 KV=8 causal."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from easydl_amd import _native  # noqa: E402

B, S, H, KV = 2, 8192, 32, 8
q = torch.randn(B, S, H, 128, device="cuda").bfloat16()
k = torch.randn(B, S, KV, 128, device="cuda").bfloat16()
v = torch.randn(B, S, KV, 128, device="cuda").bfloat16()
o = torch.empty_like(q)
lse = torch.empty(B, H, S, device="cuda")
for var in os.environ.get("VARIANTS", "0,64").split(","):
    os.environ["EDL_ATTN_FWD"] = var
    for _ in range(int(os.environ.get("ITERS", 3))):
        _native.kernels().check("edl_attn_fwd", q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(),
                                lse.data_ptr(), B, S, H, KV, 128, 1, 1 / math.sqrt(128),
                                torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
print("ok")
