"""trainer/recovery.py on the CPU tier: the memory plan of a takeover's first steps
(:func:`plan_memory`), its micro-batch pieces, and partial activation recompute."""
import torch

from easydl_amd.models.llama import Llama, get_config
from easydl_amd.trainer.recovery import RecoveryMixin, plan_memory

GB = 2**30


def test_plan_memory_enough_memory_runs_full_micro_batches():
    assert plan_memory(98 * GB, 120 * GB, 2, 32) == (1, 0)


def test_plan_memory_prefers_the_smallest_split_that_fits():
    # headline takeover (profiles/r05_ttr_headline.md): 97.8 GB needed, 68.9 GB free -> halves
    assert plan_memory(int(97.8 * GB), int(68.9 * GB), 2, 32) == (2, 0)
    assert plan_memory(100 * GB, 30 * GB, 4, 32) == (4, 0)      # 25 GB x 1.15 fits 30
    assert plan_memory(100 * GB, 60 * GB, 4, 32) == (2, 0)


def test_plan_memory_recomputes_only_as_many_layers_as_needed():
    need = int(97.8 * GB)           # 48.9 GB per sample, 56.2 GB with the margin
    split, r = plan_memory(need, 40 * GB, 2, 32)
    assert split == 2 and 0 < r < 32
    # more memory -> fewer layers recomputed; the plan's estimate fits what is free
    split2, r2 = plan_memory(need, 50 * GB, 2, 32)
    assert split2 == 2 and 0 < r2 < r
    for avail, layers in ((40 * GB, r), (50 * GB, r2)):
        est = need / 2 * 1.15 * (1 - 0.9 * layers / 32)
        assert est <= avail
    assert plan_memory(need, 1 * GB, 2, 32) == (2, 32)              # at most every layer
    assert plan_memory(need, 40 * GB, 2, 0) == (2, 0)                # no recompute knob


def test_plan_memory_counts_the_part_a_split_does_not_shrink():
    # 97.8 GB of which 14 GB stay whatever the micro-batch (transposed-weight caches): a half
    # needs 14 + 41.9 GB, not 48.9 GB -- with 60 GB free that still fits, with 55 GB it does not
    need, fixed = int(97.8 * GB), 14 * GB
    assert plan_memory(need, 68 * GB, 2, 32, fixed=fixed) == (2, 0)
    split, r = plan_memory(need, 55 * GB, 2, 32, fixed=fixed)
    assert split == 2 and r >= 1
    split0, r0 = plan_memory(need, 55 * GB, 2, 32)
    assert r > r0 or r0 == 0                                         # the fixed part costs layers


class _Host(RecoveryMixin):
    """The mixin's piece generator on its own (no trainer)."""

    def __init__(self, split, limited=False):
        self._mb_split, self._mb_limited, self._mb_plan = split, limited, (split, 0)


def test_pieces_keep_indices_and_mark_only_the_very_last():
    h = _Host(2)
    out = list(h._pieces([(0, [1, 2, 3, 4]), (1, [5, 6, 7])]))
    assert out == [(0, [1, 2], False), (0, [3, 4], False), (1, [5, 6], False), (1, [7], True)]
    h = _Host(1)
    assert list(h._pieces([(0, [1, 2]), (1, [3, 4])])) == [(0, [1, 2], False), (1, [3, 4], True)]


def test_partial_recompute_gives_the_stored_activation_gradients():
    cfg = get_config("llama-tiny", n_layers=3, dim=64, n_heads=4, n_kv_heads=2, ffn_dim=128, vocab_size=128)
    torch.manual_seed(0)
    m = Llama(cfg, device="cpu", dtype=torch.float32)
    ids = torch.randint(0, 128, (2, 16))
    grads = {}
    for rc in (False, 2, True):
        m.cfg.recompute = rc
        m.zero_grad(set_to_none=True)
        m(ids, ids).backward()
        grads[rc] = [p.grad.clone() for p in m.parameters()]
    for rc in (2, True):
        for a, b in zip(grads[False], grads[rc]):
            assert torch.allclose(a, b, atol=1e-6, rtol=1e-5)
