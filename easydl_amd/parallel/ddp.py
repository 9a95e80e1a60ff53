"""ElasticDDP: bucketed, backward-overlapped gradient all-reduce over flat buffers.

Unlike ``torch.nn.parallel.DistributedDataParallel`` the communicator can be
swapped between steps (:meth:`ElasticDDP.set_comm`) when the rendezvous epoch
changes — world size may grow or shrink without restarting the process
(SURVEY.md §2.5 P2, §3 CS2).

Mechanics:
* buckets are contiguous slices of the flat gradient buffer (no packing);
* fused ops deliver each weight gradient straight into its slice and call the
  ready callback; when every parameter of a bucket is ready the bucket's
  all-reduce is issued (strictly in bucket order, so every rank issues the
  same collective sequence) on RCCL's own stream, overlapping the rest of the
  backward;
* gradients are SUMMED; the 1/world average is folded into the optimizer's
  device-side grad scale (no extra pass);
* :meth:`no_sync` disables communication for gradient-accumulation
  micro-batches.
"""
from __future__ import annotations

import contextlib
import time
from dataclasses import dataclass, field

import torch

from easydl_amd.parallel.flat import FlatParams, _roundup


@dataclass
class Bucket:
    index: int
    group: int
    start: int
    end: int
    params: list = field(default_factory=list)
    pending: int = 0
    ready: bool = False
    seen: set = field(default_factory=set)
    view: torch.Tensor | None = None

    @property
    def numel(self) -> int:
        return self.end - self.start


class ElasticDDP:
    DEFAULT_BUCKET_MB = 128.0

    def __init__(self, flat: FlatParams, comm=None, bucket_mb: float | None = None):
        self.flat = flat
        self.comm = comm
        self.bucket_mb = bucket_mb or self.DEFAULT_BUCKET_MB
        self.sync_enabled = True
        self._works = []
        self._next = 0
        self._launch_stream = None   # collectives launched behind the side-stream weight gradients
        self.stats = {"buckets": 0, "bytes": 0, "wait_s": 0.0}
        self._build_buckets()
        flat.set_ready_callback(self._on_ready)
        self.prepare()

    # -- setup ---------------------------------------------------------------
    def _build_buckets(self) -> None:
        self.buckets: list[Bucket] = []
        self._bucket_of: dict[int, Bucket] = {}
        for gi, g in enumerate(self.flat.groups):
            cap = max(1, int(self.bucket_mb * 2**20 / g.grad.element_size()))
            cur = None
            for s in g.slots:
                if cur is None or cur.numel >= cap:
                    cur = Bucket(len(self.buckets), gi, s.offset, s.offset)
                    self.buckets.append(cur)
                cur.params.append(s.param)
                cur.end = s.offset + _roundup(s.numel)
                self._bucket_of[id(s.param)] = cur
            if cur is not None:
                cur.end = g.grad.numel()  # include trailing padding
        for b in self.buckets:
            b.view = self.flat.groups[b.group].grad[b.start:b.end]

    def set_bucket_mb(self, mb: float) -> None:
        self.bucket_mb = mb
        self._build_buckets()
        self.prepare()

    def set_comm(self, comm) -> None:
        """Swap in the communicator of a new rendezvous epoch."""
        self._works = []
        self.comm = comm
        reg = getattr(comm, "register_buffers", None)
        if reg is not None and comm.world_size > 1:
            # the xGMI engine maps every rank's flat gradient buffers once per epoch and
            # then all-reduces each bucket in place (no staging copy)
            reg([g.grad for g in self.flat.groups])
        self.prepare()

    @property
    def device(self):
        return self.flat.groups[0].grad.device if self.flat.groups else None

    @property
    def world_size(self) -> int:
        return 1 if self.comm is None else self.comm.world_size

    def _active(self) -> bool:
        return self.sync_enabled and self.comm is not None and self.comm.world_size > 1

    # -- per-step protocol -----------------------------------------------------
    def prepare(self) -> None:
        for b in self.buckets:
            b.pending = len(b.params)
            b.ready = False
            b.seen = set()
        self._next = 0
        self._works = []

    def _on_ready(self, p) -> None:
        if self.comm is not None and getattr(self.comm, "aborted", False) and self.comm.world_size > 1:
            # the epoch broke mid-backward (peer died): stop computing gradients nobody will
            # reduce; the trainer drops the step and re-forms the world
            from easydl_amd.parallel.comm import CommAborted
            raise CommAborted(f"epoch {self.comm.epoch} aborted during backward")
        if not self._active():
            return
        b = self._bucket_of.get(id(p))
        if b is None or b.ready or id(p) in b.seen:
            return
        b.seen.add(id(p))
        b.pending -= 1
        if b.pending <= 0:
            b.ready = True
            self._launch_ready()

    def _launch_ready(self) -> None:
        from easydl_amd.ops import fused
        others = fused.pending_streams(self.device) if self._next < len(self.buckets) else []
        ctx = contextlib.nullcontext()
        if others and self.buckets[self._next].ready:
            # weight gradients may still be queued on the fused ops' side stream: launch the
            # collectives from a stream that waits for the caller's stream and for those
            if self._launch_stream is None:
                from easydl_amd.utils.resources import new_stream
                self._launch_stream = new_stream(self.device)
            ls = self._launch_stream
            ls.wait_stream(torch.cuda.current_stream(self.device))
            for st in others:
                ls.wait_stream(st)
            ctx = torch.cuda.stream(ls)
        with ctx:
            self._launch_buckets()

    def _launch_buckets(self) -> None:
        while self._next < len(self.buckets) and self.buckets[self._next].ready:
            b = self.buckets[self._next]
            self._works.append(self.comm.all_reduce_async(b.view))
            self.stats["buckets"] += 1
            self.stats["bytes"] += b.view.numel() * b.view.element_size()
            self._next += 1

    def finish(self) -> None:
        """Flush every bucket (zeroing grads of unused params) and wait for the all-reduces."""
        from easydl_amd.ops import fused
        fused.join_side_streams(self.device)   # side-stream weight gradients are complete from here on
        self.flat.finalize_untouched()
        if self._active():
            for b in self.buckets:
                b.ready = True
            self._launch_ready()
            t0 = time.perf_counter()
            wait = getattr(self.comm, "wait_work", None)
            for w in self._works:
                wait(w) if wait is not None else w.wait()
            self.stats["wait_s"] += time.perf_counter() - t0
        self._works = []
        self.prepare()

    @contextlib.contextmanager
    def no_sync(self):
        prev = self.sync_enabled
        self.sync_enabled = False
        try:
            yield
        finally:
            self.sync_enabled = prev

    # -- state synchronisation -------------------------------------------------
    def broadcast_params(self, src: int = 0) -> None:
        if self.comm is None or self.comm.world_size == 1:
            return
        for g in self.flat.groups:
            self.comm.broadcast(g.data, src)
