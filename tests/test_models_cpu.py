"""Model families on CPU: forward/backward shapes, flat-param training step, loss decreases."""
import pytest
import torch

from easydl_amd.models.bert import BERT_TINY, BertMLM, SyntheticMLM
from easydl_amd.models.llama import Llama, get_config
from easydl_amd.models.mlp import MLP, SyntheticMNIST
from easydl_amd.models.resnet import ResNet, SyntheticImages
from easydl_amd.optim import FlatAdamW
from easydl_amd.parallel.flat import FlatParams


def _train(model, batch, steps=6, lr=3e-3):
    flat = FlatParams(model)
    opt = FlatAdamW(flat, lr=lr, weight_decay=0.0)
    losses = []
    for _ in range(steps):
        flat.zero_grad()
        loss = model(*batch)
        loss.backward()
        flat.finalize_untouched()
        opt.step()
        losses.append(loss.item())
    return losses


def test_llama_tiny_learns():
    torch.manual_seed(0)
    cfg = get_config("llama-tiny")
    m = Llama(cfg, dtype=torch.float32)
    ids = torch.randint(0, cfg.vocab_size, (2, 32))
    losses = _train(m, (ids, ids))
    assert losses[-1] < losses[0]


def test_bert_tiny_learns():
    torch.manual_seed(0)
    m = BertMLM(BERT_TINY, dtype=torch.float32)
    b = SyntheticMLM(BERT_TINY.vocab_size, 32).batch(range(4))
    losses = _train(m, b)
    assert losses[-1] < losses[0]


def test_resnet_small_learns():
    torch.manual_seed(0)
    m = ResNet(layers=(1, 1, 1, 1), num_classes=10, width=8)
    x, y = SyntheticImages(size=32, classes=10).batch(range(8), dtype=torch.float32)
    losses = _train(m, (x, y), steps=8)
    assert losses[-1] < losses[0]


def test_mlp_learns():
    torch.manual_seed(0)
    m = MLP()
    losses = _train(m, SyntheticMNIST(1000).batch(range(64)), steps=10)
    assert losses[-1] < losses[0] * 0.7


def test_flat_params_mixed_dtypes():
    m = ResNet(layers=(1, 1, 1, 1), num_classes=10, width=8).to(torch.bfloat16)
    for mod in m.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            mod.float()
    flat = FlatParams(m)
    names = sorted(g.name for g in flat.groups)
    assert names == ["decay", "no_decay", "no_decay_float32"], names
    assert {g.data.dtype for g in flat.groups} == {torch.bfloat16, torch.float32}


def test_flat_groups_split_under_the_byte_cap_and_train_identically():
    """Groups split at parameter boundaries into separately allocated parts of at most
    max_group_bytes of gradient (each mappable by the xGMI engine); the split changes
    nothing numerically: same losses, same final weights as one group per class."""
    cfg = get_config("llama-tiny")
    ids = torch.randint(0, cfg.vocab_size, (2, 32), generator=torch.Generator().manual_seed(3))
    out = {}
    for cap in (0, 64 << 10):
        torch.manual_seed(0)
        m = Llama(cfg, dtype=torch.float32)
        flat = FlatParams(m, max_group_bytes=cap)
        opt = FlatAdamW(flat, lr=3e-3, weight_decay=0.1)
        losses = []
        for _ in range(4):
            flat.zero_grad()
            loss = m(ids, ids)
            loss.backward()
            flat.finalize_untouched()
            opt.step()
            losses.append(loss.item())
        out[cap] = (flat, losses, torch.cat([p.detach().reshape(-1) for p in m.parameters()]))
    one, split = out[0][0], out[64 << 10][0]
    assert [g.name for g in one.groups] == ["decay", "no_decay"]
    decay_parts = [g for g in split.groups if g.name.split(".")[0] == "decay"]
    assert len(decay_parts) > 2 and decay_parts[1].name == "decay.1"
    assert all(g.grad.numel() * 4 <= (64 << 10) or len(g.slots) == 1 for g in split.groups)
    assert len({g.grad.data_ptr() for g in split.groups}) == len(split.groups)
    assert sum(g.numel for g in split.groups) == sum(g.numel for g in one.groups)
    assert all(g.weight_decay == 0.1 for g in decay_parts)
    assert out[0][1] == out[64 << 10][1]
    assert torch.equal(out[0][2], out[64 << 10][2])


def test_residual_grad_slot_accumulates_in_place():
    """gradsink.input_grad_mm: with nothing parked it is dY @ W; with a parked residual
    gradient r it returns r + dY @ W computed in place in r's storage (one GEMM, beta = 1);
    an unarmed slot is never filled by the norm, and a slot refuses a second gradient."""
    from easydl_amd.ops import gradsink
    dy, w = torch.randn(6, 4), torch.randn(4, 5)
    assert torch.allclose(gradsink.input_grad_mm(dy, w, None, (6, 5)), dy @ w)
    s = gradsink.ResidualGrad()
    assert not s.armed and s.take() is None
    r = torch.randn(6, 5)
    want = r + dy @ w
    s.arm()
    s.put(r)
    with pytest.raises(RuntimeError):
        s.put(r)
    out = gradsink.input_grad_mm(dy, w, s, (2, 3, 5))
    assert out.shape == (2, 3, 5) and out.data_ptr() == r.data_ptr()
    assert torch.allclose(out.reshape(6, 5), want, atol=1e-5)
    assert s.take() is None


def test_direct_delivery_slot_unused_next_step_is_zeroed():
    """ADVICE r3 (flat.py zero_grad): a parameter whose gradient a fused op wrote directly
    in one step but that gets no gradient in the next (unused branch) must not replay the
    stale gradient: it stays "fresh" through the backward and finalize_untouched (run by
    ElasticDDP.finish every step) zeroes it before the optimizer."""
    from easydl_amd.ops import fused, gradsink
    from easydl_amd.parallel.ddp import ElasticDDP
    from easydl_amd.parallel.flat import FlatParams

    class TwoBranch(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.a = torch.nn.Parameter(torch.randn(8, 8))
            self.b = torch.nn.Parameter(torch.randn(8, 8))

        def forward(self, x, use_a):
            return fused.linear(x, self.a if use_a else self.b).square().mean()

    m = TwoBranch()
    flat = FlatParams(m)
    ddp = ElasticDDP(flat, None)
    assert gradsink.is_flat(m.a)
    x = torch.randn(4, 8)
    flat.zero_grad()
    m(x, True).backward()
    ddp.finish()
    assert m.a.grad.abs().sum() > 0 and not flat.saw_autograd    # delivered directly, not autograd
    flat.zero_grad()
    m(x, False).backward()
    ddp.finish()
    assert torch.count_nonzero(m.a.grad) == 0 and m.b.grad.abs().sum() > 0
