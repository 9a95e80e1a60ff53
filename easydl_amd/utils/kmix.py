"""Live kernel-mix signal for the Brain (reference README.md:21-23: the Brain "monitor[s]
the performance of a training job and dynamically adjust[s] the resources").

Round 4's per-rank CU plan came only from rocprofv3 kernel-stats CSVs, which rocprofv3
writes when the profiled process EXITS: a running job never got a plan from its own kernel
mix.  Here every role measures, while it runs, how its GPU time splits between
matrix-core-bound work and bandwidth-bound work, and publishes the split with its metrics
(``metrics/<node>`` -> ``gpu_mix``), where the master's plan loop hands it to
``Planner.cu_for_profile`` exactly like a rocprof profile.

How: HIP events on the role's compute stream bracket its phases, each phase tagged with the
class of the kernels it launches -- a trainer's forward/backward micro-batches are "compute"
(GEMMs and attention on the MFMA pipes: ~90 % of that time on Llama-3-8B,
profiles/r04_final_kernel_stats.csv), its clip + fused AdamW is "memory" (HBM-bound
elementwise); a parameter server's update of its shard (AdamW / Adagrad over the shard and
the pushed rows) is "memory".  Event times are read only once the events have completed
(``query``), a step or more later: the meter never synchronises the stream.  On a CPU
device the phases are timed on the host.  It is a phase-level classification, not a
per-kernel one; rocprofv3 CSVs, when present, still take precedence.
"""
from __future__ import annotations

import time
from collections import deque
from contextlib import contextmanager

import torch

CLASSES = ("compute", "memory")


class KernelMixMeter:
    def __init__(self, device, window_s: float = 60.0):
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        self.window_s = window_s
        self._pending: deque = deque()       # (class, start event, end event, host ts)
        self._done: deque = deque()          # (host ts, class, seconds)
        self._free: list = []                # recycled events

    def _event(self):
        return self._free.pop() if self._free else torch.cuda.Event(enable_timing=True)

    @contextmanager
    def phase(self, cls: str):
        if cls not in CLASSES:
            raise ValueError(cls)
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
            self._done.append((ts, cls, s.elapsed_time(e) / 1e3))
            self._free += [s, e]
        horizon = time.time() - self.window_s
        while self._done and self._done[0][0] < horizon:
            self._done.popleft()

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
        return {"compute_frac": round(tot["compute"] / busy, 4), "memory_frac": round(tot["memory"] / busy, 4),
                "gpu_s": round(busy, 4), "phases": len(self._done), "window_s": self.window_s,
                "source": "hip-events" if self.cuda else "host-timer"}
