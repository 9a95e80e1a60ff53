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


# ---- the 8-phase kernel (kernel="nt8"): both pipelines (K % 128 == 0 -> B read-ahead; K % 128
# == 64 -> the plain 8-phase schedule), the two-tile minimum, tails of the tile pairing
@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (256, 512, 192), (512, 768, 320), (768, 256, 384),
                                   (1024, 2048, 4096), (2304, 1280, 1024), (512, 4096, 28672)])
@pytest.mark.parametrize("group_m", [4, 8])
def test_gemm_nt8_matches_fp32(cuda, M, N, K, group_m):
    from easydl_amd.ops.gemm import gemm_nt
    torch.manual_seed(M + N + K + group_m)
    a = (torch.rand(M, K, device=cuda) * 2 - 1).to(torch.bfloat16)
    b = (torch.rand(N, K, device=cuda) * 2 - 1).to(torch.bfloat16)
    c = gemm_nt(a, b, group_m=group_m, kernel="nt8")
    r = _ref(a, b)
    err = (c.float() - r).abs().max().item()
    assert err <= 1e-2 * r.abs().max().item() + 1e-2, err
    # bit-equal to the round-5 kernel (same fp32 accumulation order per output)
    assert torch.equal(c, gemm_nt(a, b, group_m=group_m))


def test_gemm_nt8_layout_and_accumulate(cuda):
    from easydl_amd.ops.gemm import gemm_nt
    M, N, K = 512, 512, 512
    a = torch.eye(M, K, device=cuda).to(torch.bfloat16)
    b = (torch.arange(N, device=cuda).float()[:, None] * 0.5 + torch.arange(K, device=cuda).float()[None, :] * 0.25)
    b = (b % 64).to(torch.bfloat16)
    assert torch.equal(gemm_nt(a, b, kernel="nt8").float(), b.float().t()[:M])
    torch.manual_seed(5)
    big_a = torch.randn(768, 640, device=cuda).to(torch.bfloat16)
    a = big_a[:, :512]
    b = torch.randn(512, 512, device=cuda).to(torch.bfloat16)
    c0 = torch.randn(768, 512, device=cuda).to(torch.bfloat16)
    c = c0.clone()
    gemm_nt(a, b, out=c, accumulate=True, kernel="nt8")
    r = c0.float() + _ref(a, b)
    assert (c.float() - r).abs().max().item() <= 1e-2 * r.abs().max().item() + 2e-2


def test_mlp_input_gradient_routes_through_nt8(cuda, monkeypatch):
    """The fused SwiGLU MLP's gate/up input gradient on the 8-phase kernel equals the hipBLASLt
    one within bf16 rounding of the same fp32 sums."""
    from easydl_amd.ops import fused, gemm
    calls = []
    real = gemm.gemm_nt
    monkeypatch.setattr(gemm, "gemm_nt", lambda *a, **k: calls.append(k.get("kernel")) or real(*a, **k))
    torch.manual_seed(11)
    x = (torch.randn(512, 512, device=cuda) * 0.5).to(torch.bfloat16)
    w_gu = (torch.randn(2048, 512, device=cuda) * 0.05).to(torch.bfloat16)
    w_dn = (torch.randn(512, 1024, device=cuda) * 0.05).to(torch.bfloat16)
    grads = {}
    for on in (False, True):
        monkeypatch.setattr(fused, "_NT8_DGRAD", on)
        xi = x.clone().requires_grad_(True)
        fused.swiglu_mlp(xi, w_gu, w_dn).float().square().mean().backward()
        grads[on] = xi.grad.float()
    ref = grads[False]
    assert calls == ["nt8"]
    assert (grads[True] - ref).abs().max().item() <= 2e-2 * ref.abs().max().item()
