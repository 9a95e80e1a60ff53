"""Host gradient shadow plumbing on the CPU tier (utils/gshadow.py, utils/vram.py helpers).

The GPU path (device -> host copies, per-group waits, pipelined restore) is covered by
tests/test_host_shadow_gpu.py; here: the segment layout a reader re-derives, the two slots'
views over one /dev/shm segment, cleanup with the job's segments, and the segment-size lookup
that keeps a tensor in a >= 2 GiB caching-allocator segment out of an IPC export."""
import os
from types import SimpleNamespace

import torch

from easydl_amd.ckpt.manager import unlink_job_segments
from easydl_amd.utils import gshadow, vram

JOB = "gshcpu"


def _groups():
    return [SimpleNamespace(grad=torch.zeros(n, dtype=dt)) for n, dt in ((1000, torch.bfloat16),
                                                                         (5000, torch.float32),
                                                                         (3, torch.bfloat16))]


def test_layout_is_aligned_and_ends_with_the_loss():
    offs, loss_off, total = gshadow.layout([2000, 20000, 6])
    assert offs == [0, 4096, 4096 + 20480] and all(o % gshadow.ALIGN == 0 for o in offs)
    assert loss_off == 4096 + 20480 + 4096 and total == loss_off + gshadow.ALIGN


def test_two_slots_round_trip_through_the_segment_and_are_unlinked_with_the_job():
    unlink_job_segments(JOB)
    gs = _groups()
    hs = gshadow.HostShadow(JOB, "worker0", gs, pin=False)
    try:
        for slot in (0, 1):
            for i, v in enumerate(hs.group_views(slot)):
                assert v.dtype == gs[i].grad.dtype and v.numel() == gs[i].grad.numel()
                v.copy_(torch.arange(v.numel()).to(v.dtype) + slot)
            hs.loss_view(slot).fill_(1.5 + slot)
        # a reader (the replacement) re-derives the layout from its own groups
        rd = gshadow.HostShadow(JOB, "worker0", _groups(), create=False, pin=False)
        for slot in (0, 1):
            for i, v in enumerate(rd.group_views(slot)):
                assert torch.equal(v, (torch.arange(v.numel()).to(v.dtype) + slot))
            assert float(rd.loss_view(slot)[0]) == 1.5 + slot
        rd.close()
        # a reader whose groups are larger refuses the segment instead of reading past it
        big = [SimpleNamespace(grad=torch.zeros(1 << 22, dtype=torch.float32))]
        try:
            gshadow.HostShadow(JOB, "worker0", big, create=False, pin=False)
            raise AssertionError("a too-small segment was accepted")
        except OSError:
            pass
    finally:
        hs.close()
        unlink_job_segments(JOB)
    assert not os.path.exists(f"/dev/shm/edl-{JOB}-gshadow-worker0")


def test_segment_lookup_finds_the_enclosing_segment():
    segs = sorted([(1 << 30, 2 << 30), (8 << 30, 64 << 20), (16 << 30, 3 << 30)])
    assert vram._segment_bytes(segs, (1 << 30) + 5) == 2 << 30
    assert vram._segment_bytes(segs, (8 << 30) + (64 << 20) - 1) == 64 << 20
    assert vram._segment_bytes(segs, (8 << 30) + (64 << 20)) == 0        # past its end
    assert vram._segment_bytes(segs, 5) == 0                             # before the first
    assert vram._segment_bytes(segs, (17 << 30)) == 3 << 30
    assert vram._segment_bytes([], 123) == 0
