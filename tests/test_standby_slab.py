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
