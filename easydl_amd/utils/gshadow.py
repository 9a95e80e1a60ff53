"""Gradient shadow in host memory: the mid-step resume's copy of the accumulated gradients when
HBM cannot hold one.

The HBM shadow (``FlatParams.ensure_shadow``) costs a second gradient buffer -- 15 GB at
Llama-3-8B.  At the headline's 2 x 8k-token micro-batches that much less HBM is left for a
replacement's first step, which then blocks behind the driver's reclaim of the dead worker's
memory (``profiles/r05_grad_shadow_ab.md``).  This shadow lives in a page-locked /dev/shm segment
instead (``/edl-<job>-gshadow-<slot>``, csrc/runtime/shm_store.cpp, one slot):

* after a micro-batch's backward the worker copies every flat gradient group device -> host on a
  side stream (the DMA engines, not the CUs), in the order the next backward writes them, and
  records one event per group; a write into a group's gradients (gradsink.is_fresh, the flat
  buffers' autograd hook) waits for that group's event, so the copy runs under the next
  micro-batch's forward and backward instead of stalling it;
* the GPU-written step marks (utils/stepmarks.py ``gstep`` / ``gmb``) bracket the copies;
* a replacement that resumes from the dead worker's HBM copies the shadow back with the pipelined
  shm -> HBM restore (ckpt/manager.py ``_restore_items``) and runs only the remaining
  micro-batches.

Two slots, written alternately: while one is being copied into (its step mark invalidated) the
other still holds the previous micro-batch's sum, so a kill during a copy loses one micro-batch,
not the step.  Layout of a slot: the groups' gradient bytes at 4 KiB-aligned offsets in group
order, then the partial loss (fp32).  A reader derives the same offsets from its own (identical)
flat groups and checks the segment size.
"""
from __future__ import annotations

import ctypes

import torch

ALIGN = 4096


def seg_name(job: str, slot: str) -> str:
    return f"/edl-{job}-gshadow-{slot}"


def layout(sizes: list[int]) -> tuple[list[int], int, int]:
    """(group offsets, loss offset, total bytes) for gradient groups of ``sizes`` bytes."""
    offs, o = [], 0
    for n in sizes:
        offs.append(o)
        o += -(-n // ALIGN) * ALIGN
    return offs, o, o + ALIGN


class HostShadow:
    def __init__(self, job: str, slot: str, groups, create: bool = True, pin: bool = True):
        from easydl_amd.ckpt.manager import ShmSegment
        self.sizes = [g.grad.numel() * g.grad.element_size() for g in groups]
        self.offsets, self.loss_off, self.total = layout(self.sizes)
        self.seg = ShmSegment(seg_name(job, slot), self.total, create=create, pin=pin, nslots=2)
        if self.seg.slot_bytes < self.total:
            self.seg.close()
            raise OSError(f"gradient shadow segment {seg_name(job, slot)}: {self.seg.slot_bytes} < {self.total} bytes")
        self.bases = [self.seg.data(0), self.seg.data(1)]
        self.pinned = self.seg.pinned
        self.dtypes = [g.grad.dtype for g in groups]

    def _host(self, slot: int, off: int, nbytes: int, dtype: torch.dtype) -> torch.Tensor:
        buf = (ctypes.c_uint8 * nbytes).from_address(self.bases[slot] + off)
        return torch.frombuffer(buf, dtype=torch.uint8).view(dtype)

    def group_views(self, slot: int) -> list[torch.Tensor]:
        return [self._host(slot, o, n, dt) for o, n, dt in zip(self.offsets, self.sizes, self.dtypes)]

    def loss_view(self, slot: int) -> torch.Tensor:
        return self._host(slot, self.loss_off, 4, torch.float32)

    def load_into(self, groups, loss_out: torch.Tensor, slot: int, stats: dict | None = None) -> None:
        """Shadow ``slot`` -> the gradient buffers and ``loss_out`` (a CUDA fp32 [1]), pipelined."""
        from easydl_amd.ckpt.manager import _restore_items
        items = [(g.grad.view(-1), o) for g, o in zip(groups, self.offsets)] + [(loss_out, self.loss_off)]
        dev = loss_out.device
        _restore_items(self.seg, slot, items, dev, torch.cuda.current_stream(dev), {} if stats is None else stats)

    def close(self, unlink: bool = False) -> None:
        self.seg.close(unlink)
