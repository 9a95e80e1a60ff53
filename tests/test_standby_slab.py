"""The standby's HBM slabs (operator/standby.py): at a takeover the slabs on the other GPUs go
back to the driver one device at a time -- never through the all-device ``empty_cache``, which
would also drop the slab the replacement's first step is about to use."""
import pytest
import torch

from easydl_amd.operator import standby


def test_takeover_releases_only_the_other_gpus_slabs(monkeypatch):
    released = []
    monkeypatch.setattr(standby, "_release_device_cache", released.append)
    monkeypatch.setattr(torch.cuda, "empty_cache", lambda: (_ for _ in ()).throw(AssertionError("all devices")))
    monkeypatch.setattr(standby, "SLABS", {0: 40 << 30, 1: 55 << 30, 2: 0, 3: 60 << 30})
    standby._release_slabs(1)
    assert released == [0, 3] and standby.SLABS == {1: 55 << 30}


@pytest.mark.gpu
def test_per_device_release_returns_cached_blocks(cuda):
    x = torch.empty(4 << 30, dtype=torch.uint8, device=cuda)
    del x
    before = torch.cuda.memory_reserved(cuda)
    assert before >= 4 << 30
    standby._release_device_cache(cuda.index or 0)
    after = torch.cuda.memory_reserved(cuda)
    assert after <= before - (4 << 30), (before, after)
    y = torch.ones(1 << 20, device=cuda)          # the allocator still works afterwards
    assert float(y.sum()) == float(1 << 20)


class _KV:
    def __init__(self, d):
        self.d = d

    def get_str(self, k):
        return self.d.get(k)

    def exists(self, k):
        return k in self.d


def test_first_workers_wait_for_a_starting_standby_replacements_do_not():
    from easydl_amd.utils import vram
    starting = _KV({"standby/roster": "", "standby/pending": "sb-0"})
    assert vram.standby_warm_on(starting, 0) is None                   # a replacement: no wait
    assert vram.standby_warm_on(starting, 0, pending=True) is False    # a first worker: wait
    assert vram.standby_warm_on(_KV({}), 0, pending=True) is None      # no standby at all
    parked = _KV({"standby/roster": "sb-0", "standby/warm/sb-0/gpu0": "{}"})
    assert vram.standby_warm_on(parked, 0) is True and vram.standby_warm_on(parked, 1, pending=True) is False


def test_warm_up_without_room_for_the_micro_batch_runs_a_short_sequence(monkeypatch):
    """(CPU) the shapes of ``_warm_llama``: the micro-batch when it fits twice over, else one
    512-token sequence at the worker's widths, else nothing."""
    spec = {"model": "llama", "batch": [4, 2048],
            "cfg": {"vocab_size": 1024, "dim": 256, "n_layers": 2, "n_heads": 4, "n_kv_heads": 2, "ffn_dim": 512,
                    "max_seq_len": 2048}}
    monkeypatch.setattr(torch.cuda, "synchronize", lambda dev=None: None)
    for free_gib, want in ((8.0, None), (4.3, 512), (4.05, 512), (3.9, False)):
        monkeypatch.setattr(torch.cuda, "mem_get_info", lambda dev=None, f=free_gib: (int(f * 2**30), 8 << 30))
        info: dict = {}
        ok = standby._warm_llama(torch.device("cpu"), spec, info)
        if want is False:
            assert not ok and "reduced_tokens" not in info
        else:
            assert ok and info.get("reduced_tokens") == want, (free_gib, info)
