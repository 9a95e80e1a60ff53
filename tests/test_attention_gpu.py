"""Hand-written flash attention vs an fp32 reference (GPU)."""

import pytest
import torch

from easydl_amd.ops.attention import attention_ref, flash_attention

pytestmark = pytest.mark.gpu


def _mk(B, S, H, KV, dev, seed, D=128):
    g = torch.Generator(device=dev).manual_seed(seed)
    q = torch.randn(B, S, H, D, device=dev, generator=g).to(torch.bfloat16).transpose(1, 2)
    k = torch.randn(B, S, KV, D, device=dev, generator=g).to(torch.bfloat16).transpose(1, 2)
    v = torch.randn(B, S, KV, D, device=dev, generator=g).to(torch.bfloat16).transpose(1, 2)
    return q, k, v


def _err(a, b):
    return ((a.float() - b.float()).abs().max() / (b.float().abs().max() + 1e-6)).item()


@pytest.mark.parametrize("B,S,H,KV,causal", [(1, 128, 4, 4, True), (2, 256, 8, 2, True), (1, 200, 4, 1, True),
                                             (1, 384, 8, 8, False), (2, 200, 4, 2, False), (1, 1024, 32, 8, True),
                                             (1, 2112, 8, 2, True), (2, 200, 8, 4, False), (2, 1000, 16, 8, True)])
@pytest.mark.parametrize("fwd", ["0", "64"])
def test_flash_attention_fwd_bwd(cuda, B, S, H, KV, causal, fwd, monkeypatch):
    """Both forward kernels (EDL_ATTN_FWD=0: 32 queries/wave; 64: software-pipelined)."""
    monkeypatch.setenv("EDL_ATTN_FWD", fwd)
    q, k, v = _mk(B, S, H, KV, cuda, S + H)
    q1, k1, v1 = (t.detach().clone().requires_grad_() for t in (q, k, v))
    o = flash_attention(q1, k1, v1, causal=causal)
    do = torch.randn_like(o)
    o.backward(do)
    q2, k2, v2 = (t.detach().float().requires_grad_() for t in (q, k, v))
    o2 = attention_ref(q2, k2, v2, causal=causal)
    o2.backward(do.float())
    assert _err(o, o2) < 2e-2, "forward"
    assert _err(q1.grad, q2.grad) < 3e-2, "dq"
    assert _err(k1.grad, k2.grad) < 3e-2, "dk"
    assert _err(v1.grad, v2.grad) < 3e-2, "dv"


@pytest.mark.parametrize("B,S,H,KV,causal", [(2, 512, 16, 16, False), (1, 200, 4, 1, True), (2, 256, 8, 2, True),
                                             (1, 1000, 8, 8, False), (1, 2112, 8, 2, True), (2, 100, 4, 4, False)])
def test_flash_attention_head_dim_64(cuda, B, S, H, KV, causal):
    """The same kernels instantiated for head dim 64 (BERT-large: 16 heads x 64, no mask)."""
    q, k, v = _mk(B, S, H, KV, cuda, S + 7 * H, D=64)
    q1, k1, v1 = (t.detach().clone().requires_grad_() for t in (q, k, v))
    o = flash_attention(q1, k1, v1, causal=causal)
    do = torch.randn_like(o)
    o.backward(do)
    q2, k2, v2 = (t.detach().float().requires_grad_() for t in (q, k, v))
    o2 = attention_ref(q2, k2, v2, causal=causal)
    o2.backward(do.float())
    assert o.shape == (B, H, S, 64)
    assert _err(o, o2) < 2e-2, "forward"
    assert _err(q1.grad, q2.grad) < 3e-2, "dq"
    assert _err(k1.grad, k2.grad) < 3e-2, "dk"
    assert _err(v1.grad, v2.grad) < 3e-2, "dv"


@pytest.mark.parametrize("fwd", ["0", "64"])
def test_flash_attention_forces_lazy_rescale(cuda, fwd, monkeypatch):
    """A late key that every query scores highly moves the running max mid-row
    (the lazy-rescale branch of both forward kernels) -- cdna_hip_programming.md rule 26."""
    monkeypatch.setenv("EDL_ATTN_FWD", fwd)
    q, k, v = _mk(1, 1000, 8, 2, cuda, 7)
    k = k.clone()
    k[:, :, 500] = q[:, 0:1, 500].expand(-1, 2, -1) * 3.0
    o = flash_attention(q, k, v, causal=True)
    ref = attention_ref(q.float(), k.float(), v.float(), causal=True)
    assert _err(o, ref) < 2e-2


@pytest.mark.parametrize("causal", [True, False])
def test_xcd_work_decode_is_bitwise_identical(cuda, causal, monkeypatch):
    """B*KV % 8 == 0: the forward and dQ kernels deal whole K/V groups to XCDs
    (EDL_ATTN_XCD, default on).  Same per-workgroup arithmetic -> identical bits."""
    q, k, v = _mk(2, 1152, 16, 4, cuda, 5)
    do = torch.randn(2, 16, 1152, 128, device=cuda).to(torch.bfloat16)
    outs = []
    for mode in ("0", "1"):
        monkeypatch.setenv("EDL_ATTN_XCD", mode)
        q1, k1, v1 = (t.detach().clone().requires_grad_() for t in (q, k, v))
        o = flash_attention(q1, k1, v1, causal=causal)
        o.backward(do)
        outs.append((o, q1.grad, k1.grad, v1.grad))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_flash_attention_speed_report(cuda):
    """Not an assertion on speed: prints TFLOP/s of fwd and fwd+bwd at the Llama-3-8B shape."""
    B, S, H, KV = 1, 8192, 32, 8
    q, k, v = _mk(B, S, H, KV, cuda, 0)
    q.requires_grad_()
    k.requires_grad_()
    v.requires_grad_()
    flops = 4 * B * H * S * S * 128 / 2
    o = flash_attention(q, k, v)
    do = torch.randn_like(o)
    for _ in range(2):
        flash_attention(q, k, v).backward(do)
    torch.cuda.synchronize()
    e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    e0.record()
    for _ in range(5):
        flash_attention(q, k, v)
    e1.record()
    for _ in range(5):
        flash_attention(q, k, v).backward(do)
    e2.record()
    torch.cuda.synchronize()
    f = e0.elapsed_time(e1) / 5
    fb = e1.elapsed_time(e2) / 5
    print(f"\n[attn] fwd {f:.3f} ms = {flops / f / 1e9:.0f} TF/s ; fwd+bwd {fb:.3f} ms = "
          f"{3.5 * flops / fb / 1e9:.0f} TF/s")


@pytest.mark.parametrize("hd", [64, 128])
def test_llama_on_hip_kernels_matches_fp32_cpu_model(cuda, hd):
    """A small Llama whose every hot op runs a HIP kernel (fused RoPE+QKV, flash attention
    at head dim 64 / 128, SwiGLU, RMSNorm, cross-entropy) against the same weights in fp32
    on the CPU reference ops: loss and gradients."""
    from easydl_amd.models.llama import Llama, get_config
    cfg = get_config("llama-tiny", dim=4 * hd, n_heads=4, n_kv_heads=2, ffn_dim=512, n_layers=2, vocab_size=512)
    torch.manual_seed(0)
    ref = Llama(cfg, device="cpu", dtype=torch.float32)
    m = Llama(cfg, device=cuda, dtype=torch.bfloat16)
    with torch.no_grad():
        for (n, p), (n2, p2) in zip(ref.named_parameters(), m.named_parameters()):
            assert n == n2
            p.copy_(p.to(torch.bfloat16).float())       # identical (bf16-representable) weights
            p2.copy_(p)
    g = torch.Generator().manual_seed(1)
    ids = torch.randint(0, cfg.vocab_size, (2, 257), generator=g)
    x, y = ids[:, :-1], ids[:, 1:]
    loss_ref = ref(x, y)
    loss_ref.backward()
    loss = m(x.to(cuda), y.to(cuda))
    loss.backward()
    assert abs(loss.item() - loss_ref.item()) / loss_ref.item() < 1e-2
    for (n, p), (_, p2) in zip(ref.named_parameters(), m.named_parameters()):
        err = ((p2.grad.float().cpu() - p.grad).norm() / p.grad.norm().clamp_min(1e-12)).item()
        assert err < 5e-2, (n, err)


@pytest.mark.parametrize("B,S,H,D,causal", [(2, 512, 16, 64, False), (1, 200, 4, 64, True), (2, 384, 8, 128, False),
                                           (1, 1000, 4, 128, True)])
@pytest.mark.parametrize("split", [False, True])
def test_packed_qkv_attention_writes_strided_gradients(cuda, B, S, H, D, causal, split, monkeypatch):
    """packed_qkv_attention (BERT: one [B*S, 3*H*D] projection in, q/k/v read by the kernels
    as row-strided slices -- or split first, EDL_ATTN_QKV_SPLIT=1 --, dq/dk/dv written
    straight into one packed gradient at row stride 3*H*D) is bitwise identical to
    flash_attention on the unpacked views, and within tolerance of the fp32 reference."""
    from easydl_amd.ops import attention
    from easydl_amd.ops.attention import packed_qkv_attention
    monkeypatch.setattr(attention, "_QKV_SPLIT", split)
    g = torch.Generator(device=cuda).manual_seed(S + H)
    qkv = torch.randn(B * S, 3 * H * D, device=cuda, generator=g).to(torch.bfloat16)
    do = torch.randn(B * S, H * D, device=cuda, generator=g).to(torch.bfloat16)
    p = qkv.clone().requires_grad_()
    o = packed_qkv_attention(p, B, S, H, causal=causal)
    assert o.shape == (B * S, H * D) and "PackedQKV" in type(o.grad_fn).__name__
    o.backward(do)
    u = qkv.clone().requires_grad_()
    q, k, v = (t.transpose(1, 2) for t in u.view(B, S, 3, H, D).unbind(2))
    ou = flash_attention(q, k, v, causal=causal).transpose(1, 2).reshape(B * S, H * D)
    ou.backward(do)
    assert torch.equal(o, ou)
    assert torch.equal(p.grad, u.grad)
    r = qkv.float().requires_grad_()
    q, k, v = (t.transpose(1, 2) for t in r.view(B, S, 3, H, D).unbind(2))
    orf = attention_ref(q, k, v, causal=causal).transpose(1, 2).reshape(B * S, H * D)
    orf.backward(do.float())
    assert _err(o, orf) < 2e-2
    for i, n in enumerate("qkv"):
        a = p.grad.view(B, S, 3, H, D)[:, :, i]
        b = r.grad.view(B, S, 3, H, D)[:, :, i]
        assert _err(a, b) < 3e-2, n
