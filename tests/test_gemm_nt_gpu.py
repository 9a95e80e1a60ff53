"""Hand-written NT GEMM (csrc/kernels/gemm_nt.hip) against an fp32 PyTorch reference."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(a, b):
    return a.float() @ b.float().t()


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (512, 768, 320), (1024, 2048, 4096), (2304, 1280, 1024)])
def test_gemm_nt_matches_fp32(cuda, M, N, K):
    from easydl_amd.ops.gemm import gemm_nt
    torch.manual_seed(M + N + K)
    a = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    b = torch.randn(N, K, device=cuda).to(torch.bfloat16)
    c = gemm_nt(a, b)
    r = _ref(a, b)
    err = (c.float() - r).abs().max().item()
    assert err <= 1e-2 * r.abs().max().item() + 1e-2, err


def test_gemm_nt_layout_with_structured_operands(cuda):
    """A = I-like selector and an asymmetric B: every output element lands at its (m, n)."""
    from easydl_amd.ops.gemm import gemm_nt
    M, N, K = 512, 512, 512
    a = torch.eye(M, K, device=cuda).to(torch.bfloat16)
    b = (torch.arange(N, device=cuda).float()[:, None] * 0.5 + torch.arange(K, device=cuda).float()[None, :] * 0.25)
    b = (b % 64).to(torch.bfloat16)
    c = gemm_nt(a, b)
    assert torch.equal(c.float(), b.float().t()[:M])


def test_gemm_nt_accumulate_and_strided_rows(cuda):
    from easydl_amd.ops.gemm import gemm_nt
    torch.manual_seed(3)
    big_a = torch.randn(768, 640, device=cuda).to(torch.bfloat16)
    a = big_a[:, :512]                      # row stride 640 > K
    b = torch.randn(512, 512, device=cuda).to(torch.bfloat16)
    c0 = torch.randn(768, 512, device=cuda).to(torch.bfloat16)
    c = c0.clone()
    gemm_nt(a, b, out=c, accumulate=True)
    r = c0.float() + _ref(a, b)
    assert (c.float() - r).abs().max().item() <= 1e-2 * r.abs().max().item() + 2e-2


def test_gemm_nt_rejects_unsupported_shapes(cuda):
    from easydl_amd.ops.gemm import gemm_nt, supported
    a = torch.randn(300, 256, device=cuda).to(torch.bfloat16)
    b = torch.randn(256, 256, device=cuda).to(torch.bfloat16)
    assert not supported(a, b)
    with pytest.raises(ValueError):
        gemm_nt(a, b)
