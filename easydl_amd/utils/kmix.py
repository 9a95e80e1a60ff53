"""Live measured signals for the Brain's per-rank CU plan (reference README.md:21-23: the
Brain "monitor[s] the performance of a training job and dynamically adjust[s] the resources").

**CU sensitivity (the primary signal, measured, no labels).**  Every ``EDL_CU_PROBE_EVERY``
steps (or when the Brain asks, runtime plan ``cu_probe``) the rank runs one step's
forward/backward on a stream confined to HALF of its CUs (``hipExtStreamCreateWithCUMask``;
utils/resources.py) instead of its own, timed with HIP events like every other step.  A kernel
mix that is matrix-core bound slows down ~2x on half the CUs; one that is HBM-bound keeps its
speed (half of the MI355X's CUs still saturate HBM).  With ``t(c) = t_C * (1 + s * (C/c - 1))``
the probe measures ``s = t_half / t_full - 1``: the share of this rank's GPU time that scales
with CUs, from its OWN kernels -- whatever code block launched them.  ``Planner.cu_for_profile``
turns ``s`` into the fewest CUs that keep the rank within a few percent of its speed.

**Phase split (secondary).**  HIP events on the compute stream also bracket the trainer's
phases -- forward/backward "compute", clip + AdamW "memory" -- giving a per-phase time split.
It is a label of where kernels were launched from, not a measurement of what they do, so the
Brain no longer plans CUs from it (it could never cut CUs for a DDP trainer).

Event times are read only once the events have completed (``query``), a step or more later:
the meter never synchronises the stream.  On a CPU device the phases are timed on the host and
there is no probe.
"""
from __future__ import annotations

import os
import statistics
import time
from collections import deque
from contextlib import contextmanager

import torch

CLASSES = ("compute", "memory")


class KernelMixMeter:
    def __init__(self, device, window_s: float = 60.0, probe_every: int | None = None):
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        self.window_s = window_s
        self._pending: deque = deque()       # (class, start event, end event, host ts)
        self._done: deque = deque()          # (host ts, class, seconds)
        self._probes: deque = deque()        # (host ts, seconds) of compute phases on half the CUs
        self._free: list = []                # recycled events
        self.probe_every = int(os.environ.get("EDL_CU_PROBE_EVERY", 0)) if probe_every is None else probe_every
        self._probe_stream = None
        self._probe_cus = (0, 0)             # (CUs of the probe stream, CUs of the rank)
        self._probe_next = False             # one probe requested (runtime plan)
        self._n_compute = 0                  # compute phases timed on the rank's own stream

    def request_probe(self) -> None:
        """Probe at the next compute phase (the Brain's ``cu_probe`` runtime knob)."""
        self._probe_next = True

    def probe_due(self, step: int) -> bool:
        """Run this step's compute phase on half the CUs?  Never the first two steps (kernel
        loads, allocator growth), and only once normal phases exist to compare against."""
        if not self.cuda or step < 2 or self._n_compute < 2:
            return False
        if self._probe_next:
            return True
        return self.probe_every > 0 and step % self.probe_every == 0

    def _half_stream(self):
        if self._probe_stream is None:
            from easydl_amd.utils import resources
            words, full = resources.half_cu_mask(self.device)
            if words is None:
                return None
            self._probe_stream = resources.masked_stream(self.device, words)
            self._probe_cus = (sum(bin(w).count("1") for w in words), full)
        return self._probe_stream

    def _event(self):
        return self._free.pop() if self._free else torch.cuda.Event(enable_timing=True)

    @contextmanager
    def phase(self, cls: str, probe: bool = False):
        """Time a phase; ``probe``: run it on a stream confined to half this rank's CUs (the
        CU-sensitivity measurement, see the module docstring)."""
        if cls not in CLASSES:
            raise ValueError(cls)
        ps = self._half_stream() if (probe and self.cuda) else None
        if ps is not None:
            self._probe_next = False
            cur = torch.cuda.current_stream(self.device)
            ps.wait_stream(cur)
            torch.cuda.set_stream(ps)
            s = self._event()
            s.record(ps)
            try:
                yield
            finally:
                e = self._event()
                e.record(ps)
                cur.wait_stream(ps)
                torch.cuda.set_stream(cur)
                self._pending.append(("probe", s, e, time.time()))
                # the probe's activations were cached under the probe stream, where the compute
                # stream's allocations cannot reuse them: hand them back to the driver
                total = torch.cuda.get_device_properties(self.device).total_memory
                if torch.cuda.memory_reserved(self.device) > 0.4 * total:
                    torch.cuda.empty_cache()
            return
        if cls == "compute":
            self._n_compute += 1
        if not self.cuda:
            t0 = time.perf_counter()
            try:
                yield
            finally:
                self._done.append((time.time(), cls, time.perf_counter() - t0))
            return
        s = self._event()
        s.record(torch.cuda.current_stream(self.device))
        try:
            yield
        finally:
            e = self._event()
            e.record(torch.cuda.current_stream(self.device))
            self._pending.append((cls, s, e, time.time()))
            if len(self._pending) > 256:      # nobody collects: keep the oldest resolved
                self.collect()

    def collect(self) -> None:
        """Resolve the phases whose end event has completed (no stream synchronisation)."""
        while self._pending and self._pending[0][2].query():
            cls, s, e, ts = self._pending.popleft()
            (self._probes.append((ts, s.elapsed_time(e) / 1e3)) if cls == "probe"
             else self._done.append((ts, cls, s.elapsed_time(e) / 1e3)))
            self._free += [s, e]
        horizon = time.time() - self.window_s
        while self._done and self._done[0][0] < horizon:
            self._done.popleft()
        while len(self._probes) > 8:
            self._probes.popleft()

    def cu_sensitivity(self) -> dict | None:
        """``{"s", "t_half_ms", "t_full_ms", "probes", "cus"}`` from the newest probes against
        the median compute phase of the window; None before a probe completed."""
        self.collect()
        full = [sec for _, c, sec in self._done if c == "compute"]
        if not self._probes or not full:
            return None
        half_cus, cus = self._probe_cus
        t_half = statistics.median(sec for _, sec in self._probes)
        t_full = statistics.median(full)
        ratio = cus / half_cus if half_cus else 2.0
        s = (t_half / t_full - 1.0) / max(1e-6, ratio - 1.0)
        return {"s": round(max(0.0, min(1.5, s)), 4), "t_half_ms": round(t_half * 1e3, 3),
                "t_full_ms": round(t_full * 1e3, 3), "probes": len(self._probes), "cus": [half_cus, cus]}

    def snapshot(self) -> dict | None:
        """``{"compute_frac", "memory_frac", "gpu_s", "phases", "source"}`` over the window, or
        None before any phase completed."""
        self.collect()
        tot = {c: 0.0 for c in CLASSES}
        for _, cls, sec in self._done:
            tot[cls] += sec
        busy = sum(tot.values())
        if busy <= 0:
            return None
        out = {"compute_frac": round(tot["compute"] / busy, 4), "memory_frac": round(tot["memory"] / busy, 4),
               "gpu_s": round(busy, 4), "phases": len(self._done), "window_s": self.window_s,
               "source": "hip-events" if self.cuda else "host-timer"}
        sens = self.cu_sensitivity()
        if sens is not None:
            out["cu_sensitivity"] = sens["s"]
            out["cu_probe"] = sens
        return out
