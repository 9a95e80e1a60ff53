"""HIP kernel numerics vs plain PyTorch fp32 references (run on the GPU box)."""
import math

import pytest
import torch
import torch.nn.functional as F

from easydl_amd.ops import fused, norms
from easydl_amd.ops.optim import adamw_flat_, grad_clip_scale

pytestmark = pytest.mark.gpu


def _close(a, b, tol):
    err = (a.float() - b.float()).abs().max().item()
    scale = b.float().abs().max().item() + 1e-6
    assert err <= tol * max(1.0, scale), f"max err {err} (scale {scale})"


@pytest.mark.parametrize("rows,cols", [(1, 64), (37, 1024), (256, 4096), (64, 8192), (5, 2056)])
@pytest.mark.parametrize("fused_res", [False, True])
def test_rmsnorm_fwd_bwd(cuda, rows, cols, fused_res):
    torch.manual_seed(0)
    x = torch.randn(rows, cols, device=cuda, dtype=torch.bfloat16, requires_grad=True)
    r = torch.randn(rows, cols, device=cuda, dtype=torch.bfloat16, requires_grad=True) if fused_res else None
    w = (1 + 0.1 * torch.randn(cols, device=cuda)).to(torch.bfloat16).requires_grad_()
    dy = torch.randn(rows, cols, device=cuda, dtype=torch.bfloat16)
    ds = torch.randn(rows, cols, device=cuda, dtype=torch.bfloat16) if fused_res else None
    if fused_res:
        y, s = norms.add_rmsnorm(x, r, w)
        (y.float() * dy.float()).sum().add_((s.float() * ds.float()).sum()).backward()
    else:
        y = norms.rmsnorm(x, w)
        (y.float() * dy.float()).sum().backward()
    gx, gw = x.grad.clone(), w.grad.clone()
    gr = r.grad.clone() if fused_res else None
    # fp32 reference
    xf = x.detach().float().requires_grad_()
    rf = r.detach().float().requires_grad_() if fused_res else None
    wf = w.detach().float().requires_grad_()
    sf = (xf + rf) if fused_res else xf
    sf_b = sf.to(torch.bfloat16).float() if fused_res else sf
    yr = sf_b * torch.rsqrt(sf_b.pow(2).mean(-1, keepdim=True) + 1e-5) * wf
    loss = (yr * dy.float()).sum()
    if fused_res:
        loss = loss + (sf * ds.float()).sum()
    loss.backward()
    _close(y, yr, 2e-2)
    _close(gx, xf.grad, 3e-2)
    _close(gw, wf.grad, 3e-2)
    if fused_res:
        _close(gr, rf.grad, 3e-2)
        _close(s, sf, 1e-2)


@pytest.mark.parametrize("rows,cols", [(33, 1024), (128, 768)])
def test_layernorm_fwd_bwd(cuda, rows, cols):
    torch.manual_seed(1)
    x = torch.randn(rows, cols, device=cuda, dtype=torch.bfloat16, requires_grad=True)
    w = (1 + 0.1 * torch.randn(cols, device=cuda)).to(torch.bfloat16).requires_grad_()
    b = (0.1 * torch.randn(cols, device=cuda)).to(torch.bfloat16).requires_grad_()
    dy = torch.randn(rows, cols, device=cuda, dtype=torch.bfloat16)
    y = norms.layernorm(x, w, b)
    (y.float() * dy.float()).sum().backward()
    xf, wf, bf = (t.detach().float().requires_grad_() for t in (x, w, b))
    yr = F.layer_norm(xf, (cols,), wf, bf, 1e-5)
    (yr * dy.float()).sum().backward()
    _close(y, yr, 2e-2)
    _close(x.grad, xf.grad, 3e-2)
    _close(w.grad, wf.grad, 3e-2)
    _close(b.grad, bf.grad, 3e-2)


@pytest.mark.parametrize("rows,F_", [(7, 64), (1024, 14336 // 4)])
def test_swiglu(cuda, rows, F_):
    torch.manual_seed(2)
    gu = torch.randn(rows, 2 * F_, device=cuda, dtype=torch.bfloat16, requires_grad=True)
    d = torch.randn(rows, F_, device=cuda, dtype=torch.bfloat16)
    o = fused.swiglu(gu)
    (o.float() * d.float()).sum().backward()
    g = gu.detach().float().requires_grad_()
    a, b_ = g.chunk(2, -1)
    orf = F.silu(a) * b_
    (orf * d.float()).sum().backward()
    _close(o, orf, 2e-2)
    _close(gu.grad, g.grad, 3e-2)


@pytest.mark.parametrize("B,S,H,KV,D", [(2, 16, 4, 2, 64), (1, 256, 32, 8, 128)])
def test_rope_qkv(cuda, B, S, H, KV, D):
    torch.manual_seed(3)
    cos, sin = fused.rope_tables(S, D, 500000.0, cuda)
    qkv = torch.randn(B * S, (H + 2 * KV) * D, device=cuda, dtype=torch.bfloat16, requires_grad=True)
    q, k, v = fused.rope_qkv(qkv, cos, sin, B, S, H, KV, D)
    assert q.shape == (B, H, S, D) and k.shape == (B, KV, S, D)
    dq, dk, dv = torch.randn_like(q), torch.randn_like(k), torch.randn_like(v)
    ((q.float() * dq.float()).sum() + (k.float() * dk.float()).sum() + (v.float() * dv.float()).sum()).backward()
    qf = qkv.detach().float().requires_grad_()
    qr, kr, vr = fused.rope_qkv_ref(qf, cos, sin, B, S, H, KV, D)
    ((qr * dq.float()).sum() + (kr * dk.float()).sum() + (vr * dv.float()).sum()).backward()
    _close(q, qr, 2e-2)
    _close(k, kr, 2e-2)
    _close(v, vr, 1e-6)
    _close(qkv.grad, qf.grad, 3e-2)


@pytest.mark.parametrize("T,V", [(4, 512), (64, 128256), (3, 1000)])
@pytest.mark.parametrize("lse", [True, False])
def test_cross_entropy(cuda, T, V, lse, monkeypatch):
    """Fused cross-entropy vs fp32 torch; the backward from the forward's saved log-sum-exp
    (default) and recomputing the row statistics (EDL_XENT_LSE=0)."""
    monkeypatch.setattr(fused, "_XENT_LSE", lse)
    torch.manual_seed(4)
    logits = (3 * torch.randn(T, V, device=cuda)).to(torch.bfloat16)
    labels = torch.randint(0, V, (T,), device=cuda)
    labels[0] = -100
    ref_in = logits.detach().float().requires_grad_()
    lr = F.cross_entropy(ref_in, labels, ignore_index=-100)
    lr.backward()
    x = logits.clone().requires_grad_()
    loss = fused.cross_entropy(x * 1, labels)  # x*1: kernel consumes a non-leaf buffer
    loss.backward()
    assert abs(loss.item() - lr.item()) < 2e-3 * max(1, abs(lr.item()))
    _close(x.grad, ref_in.grad, 2e-2)


@pytest.mark.parametrize("gdt", [torch.bfloat16, torch.float32])
def test_adamw_flat_matches_torch(cuda, gdt):
    torch.manual_seed(5)
    n = 4096 * 33
    w0 = torch.randn(n, device=cuda)
    master = w0.clone()
    p16 = w0.to(torch.bfloat16)
    m = torch.zeros(n, device=cuda)
    v = torch.zeros(n, device=cuda)
    ref = torch.nn.Parameter(w0.clone())
    opt = torch.optim.AdamW([ref], lr=1e-2, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1)
    for step in range(1, 4):
        g = torch.randn(n, device=cuda).to(gdt)
        adamw_flat_(p16, master, m, v, g, lr=1e-2, beta1=0.9, beta2=0.95, eps=1e-8, weight_decay=0.1, step=step,
                    scale=0.5)
        ref.grad = g.float() * 0.5
        opt.step()
    _close(master, ref.detach(), 1e-5)
    _close(p16, ref.detach(), 1e-2)


@pytest.mark.gpu
def test_adamw_bf16_moments_match_the_fp32_reference_and_round_like_the_cpu(cuda):
    """bf16 moments: the weights follow an fp32-moment AdamW closely (the update uses the
    unrounded moments), and the stochastically rounded m / v bits equal the CPU reference
    (ops/optim.py bf16_stochastic): the random bits are a function of (element, step)."""
    torch.manual_seed(7)
    n = 4096 * 33
    w0 = torch.randn(n, device=cuda)
    master, m, v = w0.clone(), torch.zeros(n, device=cuda, dtype=torch.bfloat16), \
        torch.zeros(n, device=cuda, dtype=torch.bfloat16)
    p16 = w0.to(torch.bfloat16)
    cm, cmm, cvv = w0.cpu().clone(), m.cpu().clone(), v.cpu().clone()
    ref = torch.nn.Parameter(w0.clone())
    opt = torch.optim.AdamW([ref], lr=1e-2, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1)
    for step in range(1, 6):
        g = torch.randn(n, device=cuda).to(torch.bfloat16)
        kw = dict(lr=1e-2, beta1=0.9, beta2=0.95, eps=1e-8, weight_decay=0.1, step=step, scale=0.5)
        adamw_flat_(p16, master, m, v, g, **kw)
        adamw_flat_(None, cm, cmm, cvv, g.cpu(), **kw)          # CPU reference of the same rounding
        ref.grad = g.float() * 0.5
        opt.step()
    _close(master, ref.detach(), 2e-3)
    # same random bits as the CPU path: equal wherever the fp32 moment agrees (the GPU contracts
    # into FMAs, so a few differ in the last fp32 bit and may round the other way)
    for a, b in ((m.cpu(), cmm), (v.cpu(), cvv)):
        ai, bi = a.view(torch.int16), b.view(torch.int16)
        assert (ai == bi).float().mean() > 0.995
        # where they differ: a few bf16 ulps apart (a 1-ulp split at one step is carried and may
        # round apart again at the next), or both next to zero with opposite signs
        tiny = 1e-3 * float(b.float().abs().max())
        near_zero = (a.float().abs() <= tiny) & (b.float().abs() <= tiny)
        ulps = (ai.int() - bi.int()).abs()
        far = (ulps > 4) & ((ai < 0) == (bi < 0)) | ((ai < 0) != (bi < 0))
        assert int((far & ~near_zero).sum()) == 0, (int((far & ~near_zero).sum()), int(ulps[~near_zero].max()))
    # master: the same wherever the moments are (elements whose moments rounded apart take a
    # slightly different step, at most a few lr)
    d = (master.cpu() - cm).abs()
    assert float((d <= 1e-6 + 1e-5 * cm.abs()).float().mean()) > 0.99
    assert float(d.max()) < 5e-2
    # deterministic: the same update from the same state gives the same bits (resume exactness)
    st = [t.clone() for t in (p16, master, m, v)]
    g = torch.randn(n, device=cuda).to(torch.bfloat16)
    kw = dict(lr=1e-2, beta1=0.9, beta2=0.95, eps=1e-8, weight_decay=0.1, step=6, scale=0.5)
    adamw_flat_(p16, master, m, v, g, **kw)
    again = [t.clone() for t in st]
    adamw_flat_(*again, g, **kw)
    assert all(torch.equal(x.view(torch.uint8), y.view(torch.uint8)) for x, y in zip((p16, master, m, v), again))


def test_grad_clip(cuda):
    torch.manual_seed(6)
    gs = [torch.randn(4096 * 7, device=cuda).to(torch.bfloat16), torch.randn(1024, device=cuda)]
    out = grad_clip_scale(gs, max_norm=1.0, pre_scale=0.5)
    norm = math.sqrt(sum(float(g.double().pow(2).sum()) for g in gs)) * 0.5
    assert abs(out[1].item() - norm) < 1e-3 * norm
    assert abs(out[0].item() - 0.5 * 1.0 / (norm + 1e-6)) < 1e-4
    assert out[2].item() == 0
    gs[1][3] = float("nan")
    out = grad_clip_scale(gs, max_norm=1.0, pre_scale=0.5)
    assert out[2].item() == 1


@pytest.mark.parametrize("n,off", [(1 << 20, 0), (1 << 20, 4), (4 * 1001, 0), (4 * 1001, 8)])
def test_sumsq_partial_matches_torch(cuda, n, off):
    """Global grad-norm partials: 16-byte path (aligned, any 4-element count) and the
    8-byte fallback (base not 16-byte aligned) both match an fp64 sum of squares."""
    from easydl_amd import _native
    k = _native.kernels()
    buf = torch.randn(n + off, device=cuda).to(torch.bfloat16)
    g = buf[off:]
    parts = torch.zeros(k("edl_sumsq_nparts", n), device=cuda)
    k.check("edl_sumsq_partial", g.data_ptr(), 0, n, parts.data_ptr(), _native.stream_of(g))
    ref = g.double().pow(2).sum().item()
    assert abs(parts.double().sum().item() - ref) <= 1e-4 * ref


def test_linear_direct_grad_into_flat(cuda):
    from easydl_amd.parallel.flat import FlatParams
    torch.manual_seed(7)
    lin = torch.nn.Linear(256, 128, bias=False).to(cuda, torch.bfloat16)
    ref_w = lin.weight.detach().float().clone().requires_grad_()
    flat = FlatParams(lin)
    x = torch.randn(64, 256, device=cuda, dtype=torch.bfloat16)
    for mb in range(2):  # two micro-batches accumulate
        y = fused.linear(x, lin.weight)
        y.float().sum().backward()
        (x.float() @ ref_w.t()).sum().backward()
    _close(lin.weight.grad, ref_w.grad, 2e-2)
    assert lin.weight.grad.data_ptr() == flat.groups[0].grad.data_ptr() + 0


@pytest.mark.parametrize("R,C", [(4096, 6144), (136, 72), (14336, 4096), (8, 200), (1000, 8)])
def test_transpose_bf16(cuda, R, C):
    from easydl_amd import _native
    x = torch.randn(R, C, device="cuda").bfloat16()
    y = torch.empty(C, R, device="cuda", dtype=torch.bfloat16)
    _native.kernels().check("edl_transpose_bf16", x.data_ptr(), y.data_ptr(), R, C, _native.stream_of(x))
    assert torch.equal(y, x.t())


@pytest.mark.parametrize("R,C", [(4096, 1024), (136, 72), (1000, 8), (16, 4104)])
def test_transpose_colsum_bf16(cuda, R, C):
    """dY^T plus fp32 column sums (the bias gradient) in one pass, vs torch."""
    from easydl_amd.ops.fused import _transposed_colsum
    x = torch.randn(R, C, device="cuda").bfloat16()
    y, part, G = _transposed_colsum(x)
    assert torch.equal(y, x.t())
    torch.testing.assert_close(part.sum(0), x.float().sum(0), rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("flat", [False, True])
def test_linear_bias_grad_from_transpose(cuda, flat):
    """Linear with bias: weight and bias gradients (NT path, bias from the fused
    transpose + column sums) match fp32, accumulated over two micro-batches."""
    from easydl_amd.parallel.flat import FlatParams
    torch.manual_seed(3)
    lin = torch.nn.Linear(1024, 3072).to(cuda, torch.bfloat16)
    rw = lin.weight.detach().float().clone().requires_grad_()
    rb = lin.bias.detach().float().clone().requires_grad_()
    if flat:
        FlatParams(lin)
    x = torch.randn(512, 1024, device=cuda, dtype=torch.bfloat16)
    for mb in range(2):
        dy = torch.randn(512, 3072, device=cuda, dtype=torch.bfloat16)
        fused.linear(x, lin.weight, lin.bias).backward(dy)
        (x.float() @ rw.t() + rb).backward(dy.float())
    _close(lin.weight.grad, rw.grad, 2e-2)
    _close(lin.bias.grad, rb.grad, 2e-2)


def test_linear_input_grad_uses_transposed_copy(cuda):
    """dX through the cached W^T (NT GEMM) equals dY @ W; the copy follows weight updates
    once a new generation starts (FlatParams.zero_grad)."""
    from easydl_amd.ops import fused
    torch.manual_seed(0)
    w = (torch.randn(512, 256, device="cuda") * 0.05).bfloat16().requires_grad_(True)
    x = torch.randn(64, 256, device="cuda").bfloat16().requires_grad_(True)
    for it in range(2):
        fused.new_weight_generation()
        y = fused.linear(x, w)
        dy = torch.randn_like(y)
        y.backward(dy)
        ref = (dy.float() @ w.detach().float())
        assert hasattr(w, "_edl_wt") and torch.equal(w._edl_wt, w.detach().t())
        torch.testing.assert_close(x.grad.float(), ref, rtol=2e-2, atol=2e-2)
        x.grad = None
        with torch.no_grad():
            w.mul_(0.5)   # "optimizer step" between generations


def test_linear_weight_grad_nt_form_matches(cuda):
    """dW through transposed activations (NT GEMM) == the TN GEMM result."""
    from easydl_amd.ops import fused
    torch.manual_seed(1)
    x = torch.randn(4096, 1024, device="cuda").bfloat16()
    w = (torch.randn(3072, 1024, device="cuda") * 0.02).bfloat16()
    dy = torch.randn(4096, 3072, device="cuda").bfloat16()
    grads = []
    for on in (True, False):
        fused._NT_WGRAD = on
        wp = w.clone().requires_grad_(True)
        fused.linear(x, wp).backward(dy)
        grads.append(wp.grad.float())
    fused._NT_WGRAD = True
    ref = dy.float().t() @ x.float()
    torch.testing.assert_close(grads[0], ref, rtol=2e-2, atol=2e-1)
    torch.testing.assert_close(grads[0], grads[1], rtol=2e-2, atol=2e-1)


@pytest.mark.parametrize("M,D,Fh", [(128, 256, 384), (200, 128, 200)])
def test_swiglu_transposed_kernels(cuda, M, D, Fh):
    """h / hT and dgu / dguT of the transposed-output SwiGLU kernels: the row-major
    outputs match the plain kernels bit for bit and the transposed ones are exact
    transposes (shapes include partial 64-tiles)."""
    from easydl_amd import _native
    k = _native.kernels()
    st = _native.stream_of
    torch.manual_seed(1)
    gu = torch.randn(M, 2 * Fh, device="cuda").bfloat16()
    dh = torch.randn(M, Fh, device="cuda").bfloat16()
    h_ref = torch.empty(M, Fh, device="cuda", dtype=torch.bfloat16)
    k.check("edl_swiglu_fwd", gu.data_ptr(), h_ref.data_ptr(), M, Fh, st(gu))
    h, hT = torch.empty_like(h_ref), torch.empty(Fh, M, device="cuda", dtype=torch.bfloat16)
    k.check("edl_swiglu_fwd_t", gu.data_ptr(), h.data_ptr(), hT.data_ptr(), M, Fh, st(gu))
    assert torch.equal(h, h_ref) and torch.equal(hT, h_ref.t())
    dgu_ref = torch.empty_like(gu)
    k.check("edl_swiglu_bwd", dh.data_ptr(), gu.data_ptr(), dgu_ref.data_ptr(), M, Fh, st(gu))
    dgu, dguT = torch.empty_like(gu), torch.empty(2 * Fh, M, device="cuda", dtype=torch.bfloat16)
    k.check("edl_swiglu_bwd_t", dh.data_ptr(), gu.data_ptr(), dgu.data_ptr(), dguT.data_ptr(), M, Fh, st(gu))
    torch.testing.assert_close(dgu.float(), dgu_ref.float(), rtol=1e-2, atol=1e-2)
    assert torch.equal(dguT, dgu.t())


def test_fused_swiglu_mlp_matches_fp32_reference(cuda):
    """swiglu_mlp (NT-form weight gradients from the transposed SwiGLU outputs) vs an
    fp32 PyTorch MLP: output, input gradient and both weight gradients."""
    from easydl_amd.ops import fused
    torch.manual_seed(2)
    M, D, Fh = 256, 256, 512
    x = torch.randn(M, D, device="cuda").bfloat16().requires_grad_(True)
    w_gu = (torch.randn(2 * Fh, D, device="cuda") * 0.05).bfloat16().requires_grad_(True)
    w_dn = (torch.randn(D, Fh, device="cuda") * 0.05).bfloat16().requires_grad_(True)
    fused.new_weight_generation()
    y = fused.swiglu_mlp(x, w_gu, w_dn)
    assert y.grad_fn is not None and "SwiGLUMLP" in type(y.grad_fn).__name__
    dy = torch.randn_like(y)
    y.backward(dy)
    xr, gr, dr = (t.detach().float().requires_grad_(True) for t in (x, w_gu, w_dn))
    g, u = (xr @ gr.t()).chunk(2, dim=-1)
    yr = (torch.nn.functional.silu(g) * u) @ dr.t()
    yr.backward(dy.float())
    for a, b in ((y, yr), (x.grad, xr.grad), (w_gu.grad, gr.grad), (w_dn.grad, dr.grad)):
        err = ((a.float() - b).abs().max() / (b.abs().max() + 1e-6)).item()
        assert err < 3e-2, err


@pytest.mark.parametrize("M,Fd", [(128, 256), (200, 136), (16, 4096)])
def test_gelu_transposed_kernels(cuda, M, Fd):
    """edl_gelu_fwd_t / edl_gelu_bwd_t vs fp32 torch GELU (tanh): h and du within bf16
    rounding, hT / duT exact transposes, column-sum partials = fp32 column sums of du."""
    from easydl_amd import _native
    k = _native.kernels()
    st = _native.stream_of
    torch.manual_seed(3)
    u = (3 * torch.randn(M, Fd, device=cuda)).bfloat16()
    dh = torch.randn(M, Fd, device=cuda).bfloat16()
    h, hT = torch.empty_like(u), torch.empty(Fd, M, device=cuda, dtype=torch.bfloat16)
    k.check("edl_gelu_fwd_t", u.data_ptr(), h.data_ptr(), hT.data_ptr(), M, Fd, st(u))
    uf = u.float().requires_grad_(True)
    hr = F.gelu(uf, approximate="tanh")
    hr.backward(dh.float())
    _close(h, hr, 1e-2)
    assert torch.equal(hT, h.t())
    G = k("edl_transpose_tiles", M)
    du, duT = torch.empty_like(u), torch.empty(Fd, M, device=cuda, dtype=torch.bfloat16)
    part = torch.empty(G, Fd, device=cuda)
    k.check("edl_gelu_bwd_t", dh.data_ptr(), u.data_ptr(), du.data_ptr(), duT.data_ptr(), part.data_ptr(), M, Fd,
            st(u))
    _close(du, uf.grad, 1e-2)
    assert torch.equal(duT, du.t())
    torch.testing.assert_close(part.sum(0), uf.grad.sum(0), rtol=1e-3, atol=1e-3 * M ** 0.5)


@pytest.mark.parametrize("flat", [False, True])
def test_fused_gelu_mlp_matches_fp32_reference(cuda, flat):
    """gelu_mlp (BERT MLP: GELU kernels emit h^T / du^T and fc1's bias column sums) vs an
    fp32 PyTorch MLP: output, input gradient, both weight and both bias gradients, with
    gradients returned to autograd or written into a flat gradient buffer (accumulated
    over two micro-batches)."""
    from easydl_amd.parallel.flat import FlatParams
    torch.manual_seed(4)
    M, D, Fd = 256, 256, 512
    mod = torch.nn.ParameterList([torch.nn.Parameter(t.bfloat16()) for t in (
        torch.randn(Fd, D, device=cuda) * 0.05, torch.randn(Fd, device=cuda) * 0.1,
        torch.randn(D, Fd, device=cuda) * 0.05, torch.randn(D, device=cuda) * 0.1)])
    pr = [p.detach().float().requires_grad_(True) for p in mod]
    if flat:
        FlatParams(mod)
    fused.new_weight_generation()
    for mb in range(2):
        x = torch.randn(M, D, device=cuda).bfloat16().requires_grad_(True)
        y = fused.gelu_mlp(x, *mod)
        assert y.grad_fn is not None and "GeluMLP" in type(y.grad_fn).__name__
        dy = torch.randn_like(y)
        y.backward(dy)
        xr = x.detach().float().requires_grad_(True)
        yr = F.linear(F.gelu(F.linear(xr, pr[0], pr[1]), approximate="tanh"), pr[2], pr[3])
        yr.backward(dy.float())
        for a, b in ((y, yr), (x.grad, xr.grad)):
            err = ((a.float() - b).abs().max() / (b.abs().max() + 1e-6)).item()
            assert err < 3e-2, err
    for p, r in zip(mod, pr):
        err = ((p.grad.float() - r.grad).abs().max() / (r.grad.abs().max() + 1e-6)).item()
        assert err < 3e-2, (tuple(p.shape), err)


@pytest.mark.parametrize("G,cols", [(1, 4), (63, 64), (65, 1000), (1024, 1024), (1100, 4096), (512, 28)])
@pytest.mark.parametrize("odt,acc", [(1, 0), (1, 1), (0, 1)])
def test_colsum_partials(cuda, G, cols, odt, acc):
    """edl_colsum (bias / norm-weight gradient from per-block partials) vs torch, every
    tail of the 64-slice x 4-chain row split, fp32 and bf16 outputs, overwrite and accumulate."""
    from easydl_amd import _native
    part = torch.randn(G, cols, device=cuda)
    dt = torch.float32 if odt == 1 else torch.bfloat16
    out = torch.randn(cols, device=cuda).to(dt)
    ref = part.double().sum(0) + (out.double() if acc else 0)
    _native.kernels().check("edl_colsum", part.data_ptr(), G, cols, out.data_ptr(), odt, acc,
                            _native.stream_of(part))
    tol = 1e-5 if odt == 1 else 1e-2
    assert ((out.double() - ref).abs().max() / ref.abs().max()).item() < tol


def test_side_stream_weight_gradients_match_compute_stream(cuda, monkeypatch):
    """Weight-gradient GEMMs on the side stream (EDL_WGRAD_STREAM) give the same flat
    gradients as on the compute stream, over two accumulated micro-batches of a small Llama,
    and reading them right after backward() is ordered after the side stream."""
    from easydl_amd.models.llama import Llama, get_config
    from easydl_amd.parallel.flat import FlatParams
    cfg = get_config("llama-tiny")
    ids = [torch.randint(0, cfg.vocab_size, (2, 128), device=cuda) for _ in range(2)]
    grads = []
    for on in (False, True):
        monkeypatch.setattr(fused, "_WGRAD_STREAM", on)
        torch.manual_seed(0)
        m = Llama(cfg, device=cuda, dtype=torch.bfloat16)
        flat = FlatParams(m)
        flat.zero_grad()
        fused.new_weight_generation()
        for x in ids:
            m(x, x).backward()
        grads.append(torch.cat([g.grad.float().clone() for g in flat.groups]))
    err = ((grads[0] - grads[1]).abs().max() / grads[0].abs().max()).item()
    assert err < 1e-2, err   # same GEMMs on another stream; an ordering race shows as O(1) errors


@pytest.mark.parametrize("side", [False, True])
@pytest.mark.parametrize("flat", [False, True])
def test_bert_layer_residual_grad_slots_match_fp32(cuda, flat, side, monkeypatch):
    """A post-LN BERT layer on the HIP kernels, where the input's two gradients (the qkv /
    fc1 GEMM input gradient and LayerNorm's residual gradient) are summed in the GEMM
    epilogue (gradsink.ResidualGrad, addmm_ with beta = 1) instead of an add kernel, vs the
    same layer in fp32 on the CPU: input gradient and every parameter gradient, over two
    accumulated micro-batches; both slots are used."""
    from easydl_amd.models.bert import BertConfig, BertLayer
    from easydl_amd.ops import gradsink
    from easydl_amd.parallel.flat import FlatParams
    used = []
    orig = gradsink.input_grad_mm

    def counting(dy2, w, slot, shape):
        used.append(slot is not None and slot.g is not None)
        return orig(dy2, w, slot, shape)
    monkeypatch.setattr(gradsink, "input_grad_mm", counting)
    # side: weight gradients on the side stream (EDL_WGRAD_STREAM=1) -- the parked residual
    # gradient is also what fc2 / wo's side-stream weight GEMM reads
    monkeypatch.setattr(fused, "_WGRAD_STREAM", side)
    torch.manual_seed(5)
    c = BertConfig(vocab_size=512, dim=256, n_layers=1, n_heads=4, ffn_dim=1024, max_pos=128)
    layer = BertLayer(c, cuda, torch.bfloat16)
    with torch.no_grad():
        for p in layer.parameters():
            p.add_(0.05 * torch.randn_like(p))
    ref = BertLayer(c, "cpu", torch.float32)
    ref.load_state_dict({k: v.float().cpu() for k, v in layer.state_dict().items()})
    if flat:
        FlatParams(layer)
    fused.new_weight_generation()
    B, S = 2, 128
    for mb in range(2):
        x = torch.randn(B * S, c.dim, device=cuda).bfloat16().requires_grad_(True)
        y = layer(x, B, S)
        dy = torch.randn_like(y)
        y.backward(dy)
        xr = x.detach().float().cpu().requires_grad_(True)
        yr = ref(xr, B, S)
        yr.backward(dy.float().cpu())
        _close(y.cpu(), yr, 3e-2)
        _close(x.grad.cpu(), xr.grad, 3e-2)
    assert sum(used) == 4, used   # qkv + fc1 input gradients took their slot, per micro-batch
    for (n, p), r in zip(layer.named_parameters(), ref.parameters()):
        err = ((p.grad.float().cpu() - r.grad).abs().max() / (r.grad.abs().max() + 1e-6)).item()
        assert err < 3e-2, (n, err)


@pytest.mark.parametrize("M,N,J", [(1000, 128, 256), (2048, 1024, 1024), (4096, 256, 512), (96, 384, 768),
                                   (16384, 128, 256), (1000, 4096, 4096), (160, 8192, 2048),
                                   (8192, 1024, 1024)])
@pytest.mark.parametrize("out_dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("acc", [False, True])
def test_gemm_tn_matches_fp32(cuda, M, N, J, out_dt, acc):
    """edl_gemm_tn (dW = dY^T X from the row-major operands via transposing LDS reads) vs
    fp32 torch: row tails (M % 32 != 0), the split-M partial-slab path, the 256 x 256 kernel
    (>= 256 output tiles), bf16 / fp32 outputs, overwrite and accumulate."""
    torch.manual_seed(6)
    dy = torch.randn(M, N, device=cuda).bfloat16()
    x = torch.randn(M, J, device=cuda).bfloat16()
    out = torch.randn(N, J, device=cuda).to(out_dt)
    ref = dy.float().t() @ x.float() + (out.float() if acc else 0)
    fused.gemm_tn(dy, x, out=out, accumulate=acc)
    err = ((out.float() - ref).abs().max() / ref.abs().max()).item()
    assert err < (1e-2 if out_dt == torch.bfloat16 else 1e-4), err


@pytest.mark.parametrize("M,C", [(16384, 1024), (1000, 64), (40, 4096), (16384, 3072), (777, 512), (5000, 2056)])
def test_colsum_bf16_partials(cuda, M, C):
    """Bias-gradient column sums of a bf16 [M, C] matrix (edl_colsum_bf16_partial + edl_colsum)."""
    from easydl_amd import _native
    t = torch.randn(M, C, device=cuda).bfloat16()
    part, G = fused._colsum_partial(t)
    out = torch.empty(C, device=cuda)
    _native.kernels().check("edl_colsum", part.data_ptr(), G, C, out.data_ptr(), 1, 0, _native.stream_of(t))
    torch.testing.assert_close(out, t.float().sum(0), rtol=1e-4, atol=1e-3 * M ** 0.5)


@pytest.mark.parametrize("G,C", [(1024, 1024), (1000, 4096), (512, 3072), (37, 8192), (1024, 16384), (7, 260),
                                 (33, 4100)])
@pytest.mark.parametrize("odt,acc", [(1, 0), (1, 1), (0, 1)])
def test_colsum_block_widths(cuda, G, C, odt, acc):
    """edl_colsum on slabs whose width picks each column-group block shape (16/8/4/2/1
    groups of 4 per block), a ragged last block and G not a multiple of the slice count."""
    from easydl_amd import _native
    part = torch.randn(G, C, device=cuda)
    dt = torch.float32 if odt else torch.bfloat16
    out = torch.randn(C, device=cuda).to(dt)
    want = part.sum(0) + (out.float() if acc else 0)
    _native.kernels().check("edl_colsum", part.data_ptr(), G, C, out.data_ptr(), odt, acc, _native.stream_of(part))
    tol = 1e-4 * G ** 0.5 if odt else 2e-2 * G ** 0.5
    torch.testing.assert_close(out.float(), want, rtol=1e-4 if odt else 1e-2, atol=tol)


def test_wt_cache_batched_refresh(cuda, monkeypatch):
    """The cached transposed weights of a new generation are refreshed together in one
    edl_transpose_bf16_multi launch (ragged tile counts, rows/cols not multiples of 128)
    and equal the transposes of the mutated weights; the per-weight path agrees."""
    monkeypatch.setattr(fused, "_WT_ALL", [])
    monkeypatch.setattr(fused, "_WT_DESC", {})
    ws = [torch.randn(r, c, device=cuda).bfloat16() for r, c in ((384, 512), (1000, 24), (256, 1032), (8, 8))]
    fused.new_weight_generation()
    for w in ws:
        torch.testing.assert_close(fused._wt_of(w), w.t(), rtol=0, atol=0)
    for batch in (True, False):
        monkeypatch.setattr(fused, "_WT_BATCH", batch)
        for w in ws:
            w.mul_(-2).add_(1)   # parameter mutation between steps
        fused.new_weight_generation()
        fused._wt_of(ws[1])      # first use: every stale copy refreshed (one launch when batched)
        assert all(w._edl_wt_gen == fused._WT_GEN[0] for w in ws) == batch
        for w in ws:
            torch.testing.assert_close(fused._wt_of(w), w.t(), rtol=0, atol=0)


@pytest.mark.parametrize("tn", ["0", "1"])
def test_linear_bias_wgrad_tn_and_nt_match_fp32(cuda, tn, monkeypatch):
    """A biased linear layer's weight / bias gradients through the TN kernel (no transposes)
    and through the NT form on transposed copies, flat buffers, two micro-batches."""
    from easydl_amd.parallel.flat import FlatParams
    monkeypatch.setattr(fused, "_WGRAD_TN", tn)
    torch.manual_seed(7)
    mod = torch.nn.ParameterList([torch.nn.Parameter((torch.randn(384, 512, device=cuda) * 0.05).bfloat16()),
                                  torch.nn.Parameter((torch.randn(384, device=cuda) * 0.1).bfloat16())])
    pr = [p.detach().float().requires_grad_(True) for p in mod]
    FlatParams(mod)
    fused.new_weight_generation()
    for mb in range(2):
        x = torch.randn(1024, 512, device=cuda).bfloat16().requires_grad_(True)
        y = fused.linear(x, mod[0], mod[1])
        dy = torch.randn_like(y)
        y.backward(dy)
        F.linear(x.detach().float(), pr[0], pr[1]).backward(dy.float())
    for p, r in zip(mod, pr):
        err = ((p.grad.float() - r.grad).abs().max() / (r.grad.abs().max() + 1e-6)).item()
        assert err < 2e-2, (tuple(p.shape), err)


def test_swiglu_mlp_mixed_weight_gradient_forms_match_fp32(cuda, monkeypatch):
    """SwiGLU MLP whose two weight gradients take different forms under the auto policy with
    EDL_WGRAD_TN_WIDE_J = 8192: the down projection (input width 8448) on the TN kernel from h,
    the big gate/up one as hipBLASLt NT on d(gate_up)^T; output, input and weight gradients vs fp32."""
    from easydl_amd.parallel.flat import FlatParams
    monkeypatch.setattr(fused, "_WGRAD_TN_WIDE", 8192)
    torch.manual_seed(10)
    M, D, Fh = 256, 512, 8448
    assert fused._tn_dims(torch.empty(1, device=cuda, dtype=torch.bfloat16), D, Fh)          # down: TN
    assert not fused._tn_dims(torch.empty(1, device=cuda, dtype=torch.bfloat16), 2 * Fh, D)  # gate/up: NT
    mod = torch.nn.ParameterList([torch.nn.Parameter((torch.randn(2 * Fh, D, device=cuda) * 0.03).bfloat16()),
                                  torch.nn.Parameter((torch.randn(D, Fh, device=cuda) * 0.02).bfloat16())])
    pr = [p.detach().float().requires_grad_(True) for p in mod]
    FlatParams(mod)
    fused.new_weight_generation()
    x = torch.randn(M, D, device=cuda).bfloat16().requires_grad_(True)
    y = fused.swiglu_mlp(x, mod[0], mod[1])
    dy = torch.randn_like(y)
    y.backward(dy)
    xr = x.detach().float().requires_grad_(True)
    g, u = (xr @ pr[0].t()).chunk(2, dim=-1)
    yr = (F.silu(g) * u) @ pr[1].t()
    yr.backward(dy.float())
    for a, b in ((y, yr), (x.grad, xr.grad), (mod[0].grad, pr[0].grad), (mod[1].grad, pr[1].grad)):
        err = ((a.float() - b).abs().max() / (b.abs().max() + 1e-6)).item()
        assert err < 3e-2, err
