"""Gradient precision: bf16 vs fp32 flat gradient buffers (ElasticTrainer(grad_dtype=...),
bench.py --grad-dtype).

* fp32 buffers take the weight gradients straight from hipBLASLt's bf16 x bf16 -> fp32
  GEMMs (gradsink.write_mm: mm / addmm ``dtype_out``, beta = 1 across micro-batches) and
  from the fused kernels' fp32 outputs: after two accumulated micro-batches they are
  closer to an fp32 reference than the bf16 buffers;
* a ~200-step loss-parity run of a small Llama (4 accumulated micro-batches per step, the
  headline's accumulation depth) with either dtype: the two loss curves agree.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _model(cuda, seed=0):
    from easydl_amd.models.llama import Llama, get_config
    torch.manual_seed(seed)
    cfg = get_config("llama-tiny")
    return cfg, Llama(cfg, device=cuda, dtype=torch.bfloat16)


def _batch(cfg, cuda, step, mb, B=4, S=128):
    # a learnable stream: every sequence is an arithmetic progression mod V with a random stride
    g = torch.Generator().manual_seed(1000 * step + mb)
    start = torch.randint(0, cfg.vocab_size, (B, 1), generator=g)
    stride = torch.randint(1, 8, (B, 1), generator=g)
    ids = (start + stride * torch.arange(S)) % cfg.vocab_size
    return ids.to(cuda)


def test_fp32_grad_buffers_are_closer_to_fp32_reference(cuda):
    from easydl_amd.parallel.flat import FlatParams
    cfg, ref_m = _model(cuda)
    ref = {n: torch.zeros_like(p, dtype=torch.float32) for n, p in ref_m.named_parameters()}
    ids = [_batch(cfg, cuda, 0, mb) for mb in range(4)]
    # reference: each micro-batch's bf16-computed gradient summed in fp64 (the exact sum of the
    # same per-micro-batch products both buffers accumulate)
    for x in ids:
        ref_m.zero_grad(set_to_none=True)
        ref_m(x, x).backward()
        for n, p in ref_m.named_parameters():
            ref[n] += p.grad.double().float() if p.grad is not None else 0
    errs = {}
    for gdt in (None, torch.float32):
        cfg, m = _model(cuda)
        flat = FlatParams(m, grad_dtype=gdt)
        flat.zero_grad()
        for x in ids:
            m(x, x).backward()
        flat.finalize_untouched()
        torch.cuda.synchronize()
        num = den = 0.0
        for n, p in m.named_parameters():
            num += float((p.grad.float() - ref[n]).norm()) ** 2
            den += float(ref[n].norm()) ** 2
        errs["bf16" if gdt is None else "fp32"] = (num / den) ** 0.5
        assert flat.groups[0].grad.dtype == (gdt or torch.bfloat16)
    assert errs["fp32"] < errs["bf16"], errs
    assert errs["fp32"] < 2e-2, errs


@pytest.mark.timeout(300)
def test_loss_parity_bf16_vs_fp32_grad_accumulation(cuda):
    from easydl_amd.optim import FlatAdamW
    from easydl_amd.parallel.flat import FlatParams
    curves = {}
    for name, gdt in (("bf16", None), ("fp32", torch.float32)):
        cfg, m = _model(cuda)
        flat = FlatParams(m, weight_decay=0.1, grad_dtype=gdt)
        opt = FlatAdamW(flat, lr=2e-3)
        losses = []
        for step in range(200):
            flat.zero_grad()
            tot = 0.0
            for mb in range(4):
                x = _batch(cfg, cuda, step, mb)
                loss = m(x, x) * 0.25
                loss.backward()
                tot += float(loss.detach())
            flat.finalize_untouched()
            opt.step()
            losses.append(tot)
        curves[name] = losses
    a, b = torch.tensor(curves["bf16"]), torch.tensor(curves["fp32"])
    # both learn the progressions ...
    assert a[-20:].mean() < 0.5 * a[:5].mean() and b[-20:].mean() < 0.5 * b[:5].mean(), (a[-5:], b[-5:])
    # ... along the same curve (late-training gap well under the loss itself)
    gap = (a[-50:] - b[-50:]).abs().mean() / b[-50:].mean()
    print(f"loss bf16 {a[-10:].mean():.4f} fp32 {b[-10:].mean():.4f} rel gap (last 50) {gap:.4f}")
    assert gap < 0.1, gap
