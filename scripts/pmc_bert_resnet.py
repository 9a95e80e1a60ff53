"""Run the BERT-large and ResNet-50 hand-written hot kernels a few times at their
production shapes, for rocprofv3 --pmc passes (scripts/gpu_pmc_bert_resnet.sh): the
GELU MLP kernels (16384 x 4096), the packed-qkv split and head-dim-64 attention
(B 32, S 512, 16 heads), and the channels-last BatchNorm forward / backward at the
widest ResNet-50 activations (256 x 56 x 56 x 256 with residual, x 64 without)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from easydl_amd import _native  # noqa: E402
from easydl_amd.ops.attention import packed_qkv_attention  # noqa: E402
from easydl_amd.ops.batchnorm import bn_act  # noqa: E402

dev = torch.device("cuda", 0)
k = _native.kernels()
st = _native.stream_of
M, Fd = 16384, 4096
u = torch.randn(M, Fd, device=dev).bfloat16()
dh = torch.randn(M, Fd, device=dev).bfloat16()
h, hT = torch.empty_like(u), torch.empty(Fd, M, device=dev, dtype=torch.bfloat16)
du, duT = torch.empty_like(u), torch.empty(Fd, M, device=dev, dtype=torch.bfloat16)
part = torch.empty(k("edl_transpose_tiles", M), Fd, device=dev)
for _ in range(3):
    k.check("edl_gelu_fwd_t", u.data_ptr(), h.data_ptr(), hT.data_ptr(), M, Fd, st(u))
    k.check("edl_gelu_bwd_t", dh.data_ptr(), u.data_ptr(), du.data_ptr(), duT.data_ptr(), part.data_ptr(), M, Fd,
            st(u))
del u, dh, h, hT, du, duT, part
B, S, H, D = 32, 512, 16, 64
qkv = torch.randn(B * S, 3 * H * D, device=dev).bfloat16().requires_grad_()
do = torch.randn(B * S, H * D, device=dev).bfloat16()
for _ in range(3):
    packed_qkv_attention(qkv, B, S, H, causal=False).backward(do)
del qkv, do
for C, res in ((256, True), (64, False)):
    bn = torch.nn.BatchNorm2d(C).to(dev)
    x = torch.randn(256, C, 56, 56, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
    x.requires_grad_()
    r = torch.randn_like(x) if res else None
    dz = torch.randn_like(x)
    for _ in range(3):
        bn_act(x, bn, residual=r, relu=True).backward(dz)
    del bn, x, r, dz
torch.cuda.synchronize()
print("pmc driver done")
