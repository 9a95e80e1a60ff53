"""Run each hand-written hot kernel a few times at its production shape, for
rocprofv3 --pmc passes (scripts/gpu_pmc.sh): fused AdamW over 1e9 params,
the bf16 transpose, flash-attention fwd/bwd (Llama-3-8B 8k shape), RMSNorm
fwd/bwd, SwiGLU, the 128k-vocab cross-entropy and the snapshot checksum."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["EDL_ATTN"] = "hip"
from easydl_amd import _native  # noqa: E402
from easydl_amd.ckpt.manager import checksum_tensor  # noqa: E402
from easydl_amd.ops import fused, norms  # noqa: E402
from easydl_amd.ops.attention import flash_attention  # noqa: E402
from easydl_amd.ops.optim import adamw_flat_  # noqa: E402

dev = torch.device("cuda", 0)
k = _native.kernels()
n = 1 << 30
p16 = torch.zeros(n, device=dev, dtype=torch.bfloat16)
w, m, v = (torch.zeros(n, device=dev) for _ in range(3))
g = torch.zeros(n, device=dev, dtype=torch.bfloat16)
for i in range(3):
    adamw_flat_(p16, w, m, v, g, lr=1e-4, beta1=0.9, beta2=0.95, eps=1e-8, weight_decay=0.1, step=i + 1)
del w, m, v
acc = torch.zeros(1, dtype=torch.int64, device=dev)
for _ in range(3):
    checksum_tensor(p16, acc)
wt = torch.empty(4096, 14336, device=dev, dtype=torch.bfloat16)
src = p16[:14336 * 4096].view(14336, 4096)
for _ in range(3):
    k.check("edl_transpose_bf16", src.data_ptr(), wt.data_ptr(), 14336, 4096, _native.stream_of(src))
del p16, g, wt
B, S, H, KV = 1, 8192, 32, 8
q = torch.randn(B, S, H, 128, device=dev, dtype=torch.bfloat16).transpose(1, 2).requires_grad_()
kk = torch.randn(B, S, KV, 128, device=dev, dtype=torch.bfloat16).transpose(1, 2).requires_grad_()
vv = torch.randn(B, S, KV, 128, device=dev, dtype=torch.bfloat16).transpose(1, 2).requires_grad_()
do = torch.randn(B, H, S, 128, device=dev, dtype=torch.bfloat16)
for _ in range(3):
    flash_attention(q, kk, vv).backward(do)
x = torch.randn(16384, 4096, device=dev, dtype=torch.bfloat16, requires_grad=True)
gw = torch.ones(4096, device=dev, dtype=torch.bfloat16, requires_grad=True)
for _ in range(3):
    norms.rmsnorm(x, gw, 1e-5).sum().backward()
gu = torch.randn(16384, 2 * 14336, device=dev, dtype=torch.bfloat16, requires_grad=True)
for _ in range(3):
    fused.swiglu(gu).sum().backward()
logits = torch.randn(16384, 128256, device=dev, dtype=torch.bfloat16)
labels = torch.randint(0, 128256, (16384,), device=dev)
for _ in range(3):
    fused.cross_entropy(logits.clone(), labels)
torch.cuda.synchronize()
print("ok")
