"""Step marks: which optimizer update the HBM state of a worker slot has finished.

One 4 KiB shm page per worker slot (``/edl-<job>-marks-<role><index>``), written by the
worker's GPU in stream order (``edl_ps_signal`` kernel, system-scope store into the page,
page-locked and device-mapped), read by the process that replaces it:

* ``begin`` = the step whose update is about to start (written before the optimizer kernels),
* ``done``  = the step whose update has finished (written after them),
* ``pid``   = the writer,
* ``gstep``, ``gmb`` (one pair per shadow slot, 2 slots) = that slot of the gradient shadow
  (``FlatParams.ensure_shadow`` in HBM: slot 0 only; utils/gshadow.py in host memory: the two
  slots alternate) holds the summed gradients of micro-batches ``[0, gmb)`` of step ``gstep``;
  ``gmb = 0``: not valid.  A slot is copied on a side stream after a micro-batch's backward,
  between an invalidating write (``gmb = 0``) and its mark, so a kill in the middle of the copy
  leaves ``gmb = 0`` there -- and the other host slot still holds the previous micro-batch.

When a worker is SIGKILLed, its GPU queues stop (utils/procfs.py).  If ``begin == done == K``
no update was in flight, so the weights, fp32 master and moments in its HBM are exactly the
state after step K.  A replacement that adopted that HBM (utils/vram.py) then resumes from
step K without restoring a snapshot: no host -> HBM copy, no lost steps, and the same
per-step seeds as an uninterrupted run.  With ``begin != done`` it restores from /dev/shm.  When the
shadow also names step K + 1, the replacement copies it into its gradient buffers and runs
only the micro-batches of step K + 1 the dead worker had not finished (a mid-step resume).

Reference: the reference's recovery contract ("resume the training" after a failure,
/root/reference/README.md:25-29); the mechanism is ours.
"""
from __future__ import annotations

import ctypes
import os

import torch

from easydl_amd import _native

BEGIN, DONE, PID, GSTEP, GMB = 0, 4, 8, 16, 20     # byte offsets in the page (GSTEP/GMB: + 8 per slot)


def best_shadow(marks: tuple, step: int) -> tuple[int, int] | None:
    """(shadow slot, micro-batches) of the fullest valid shadow of ``step`` among the
    (gstep, gmb) pairs ``marks`` = (gstep0, gmb0, gstep1, gmb1); None if none is."""
    ok = [(marks[2 * s + 1], s) for s in range(len(marks) // 2) if marks[2 * s + 1] and marks[2 * s] == step]
    if not ok:
        return None
    mb, s = max(ok)
    return s, mb


def page_name(job: str, slot: str) -> str:
    return f"/edl-{job}-marks-{slot}"


class StepMarks:
    def __init__(self, job: str, slot: str, create: bool = True, device: torch.device | None = None):
        self.name = page_name(job, slot)
        self.rt = _native.runtime()
        host, dev = ctypes.c_void_p(), ctypes.c_void_p()
        pin = device is not None and device.type == "cuda"
        self.h = self.rt("edl_mark_open", self.name.encode(), 1 if create else 0, 1 if pin else 0,
                         ctypes.byref(host), ctypes.byref(dev))
        if not self.h:
            raise OSError(f"cannot open step-mark page {self.name}")
        self.host = host.value
        self.dev = dev.value            # None: written from the host (CPU training / not pinned)
        self.device = device

    def _u32(self, off: int):
        return ctypes.c_uint32.from_address(self.host + off)

    def set_now(self, step: int) -> None:
        """Host write of begin = done = ``step`` (no update in flight; the stream is idle)."""
        self._u32(BEGIN).value = step & 0xFFFFFFFF
        self._u32(DONE).value = step & 0xFFFFFFFF
        self._u32(GMB).value = 0
        self._u32(GMB + 8).value = 0
        ctypes.c_int64.from_address(self.host + PID).value = os.getpid()

    def _mark(self, off: int, step: int, stream) -> None:
        if self.dev is not None:
            _native.kernels().check("edl_ps_signal", self.dev + off, step & 0xFFFFFFFF,
                                    stream.cuda_stream if stream is not None else None)
        else:
            self._u32(off).value = step & 0xFFFFFFFF

    def begin(self, step: int, stream=None) -> None:
        self._mark(BEGIN, step, stream)

    def done(self, step: int, stream=None) -> None:
        self._mark(DONE, step, stream)

    def shadow(self, step: int, mb: int, stream=None, slot: int = 0) -> None:
        """Gradient shadow ``slot``: ``mb`` = 0 before a copy starts, then (``step``, ``mb``) after it."""
        if mb:
            self._mark(GSTEP + 8 * slot, step, stream)
        self._mark(GMB + 8 * slot, mb, stream)

    def read(self) -> tuple[int, int, int]:
        return (self._u32(BEGIN).value, self._u32(DONE).value,
                ctypes.c_int64.from_address(self.host + PID).value)

    def read_shadow(self, slot: int = 0) -> tuple[int, int]:
        """(gstep, gmb) of gradient-shadow ``slot``."""
        return self._u32(GSTEP + 8 * slot).value, self._u32(GMB + 8 * slot).value

    def close(self, unlink: bool = False) -> None:
        if self.h:
            self.rt("edl_mark_close", self.h, 1 if unlink else 0)
            self.h = None


def read_slot(job: str, slot: str, shadow: bool = False) -> tuple | None:
    """(begin, done, pid) of a slot's page -- plus (gstep0, gmb0, gstep1, gmb1) with ``shadow``
    -- or None if there is none."""
    try:
        m = StepMarks(job, slot, create=False)
    except OSError:
        return None
    try:
        return m.read() + ((m.read_shadow(0) + m.read_shadow(1)) if shadow else ())
    finally:
        m.close()
