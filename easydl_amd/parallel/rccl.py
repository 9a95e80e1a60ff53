"""Native RCCL data plane (csrc/runtime/rccl_comm.cpp).

:class:`RcclComm` is one rank's RCCL communicator for one epoch / group:

* bootstrap through the job's store: rank 0 draws the ``ncclUniqueId`` and
  publishes it under ``<prefix>/rccl_id``; the others read it;
* creation is non-blocking inside RCCL and polled by the native layer with the
  GIL released; :meth:`abort` (watchdog thread) or the deadline abandons it —
  a rank never stays stuck building a communicator with a dead peer;
* collectives run on a dedicated high-priority HIP stream ordered after the
  caller's stream, and return a work handle whose ``wait()`` orders the
  caller's stream after the collective (the same contract as a
  ``ProcessGroupNCCL`` work object, so ElasticDDP overlaps it with backward);
* :meth:`shrink` drops dead ranks without a full re-init where the loaded RCCL
  has ``ncclCommShrink``.

Selected with ``EDL_COMM=native`` (``Communicator(data_backend="native")``);
the default data plane stays ``ProcessGroupNCCL``.
"""
from __future__ import annotations

import ctypes
import time

import torch
import torch.distributed as dist

from easydl_amd import _native

_DT = {torch.int8: 0, torch.uint8: 1, torch.int32: 2, torch.int64: 4, torch.float16: 6, torch.float32: 7,
       torch.float64: 8, torch.bfloat16: 9}
_OP = {dist.ReduceOp.SUM: 0, dist.ReduceOp.PRODUCT: 1, dist.ReduceOp.MAX: 2, dist.ReduceOp.MIN: 3,
       dist.ReduceOp.AVG: 4}


class RcclError(RuntimeError):
    pass


def available() -> tuple[bool, int, bool]:
    """(RCCL resolvable, version, ncclCommShrink present)."""
    v, s = ctypes.c_int(0), ctypes.c_int(0)
    ok = _native.runtime()("edl_rccl_available", ctypes.byref(v), ctypes.byref(s))
    return bool(ok), v.value, bool(s.value)


def _err(rc: int) -> str:
    msg = _native.runtime()("edl_rccl_error_string", rc)
    return (msg or b"?").decode()


class _Work:
    def __init__(self, event: torch.cuda.Event, keep):
        self._event, self._keep = event, keep

    def wait(self, *a, **k):
        torch.cuda.current_stream().wait_event(self._event)
        self._keep = None
        return True

    def is_completed(self):
        return self._event.query()


class RcclComm:
    def __init__(self, store, prefix: str, rank: int, world: int, device: torch.device, timeout_s: float = 120.0):
        self.rank, self.world_size = rank, world
        self.device = torch.device(device)
        self._rt = _native.runtime()
        self._abort_flag = ctypes.c_int(0)
        self._h = None
        self._aborted = False
        key = f"{prefix}/rccl_id"
        idbuf = ctypes.create_string_buffer(128)
        if rank == 0:
            rc = self._rt("edl_rccl_unique_id", idbuf)
            if rc != 0:
                raise RcclError(f"ncclGetUniqueId failed: {_err(rc)}")
            store.set(key, idbuf.raw)
        else:
            raw = store.get(key)  # TCPStore.get waits for the key (store timeout)
            ctypes.memmove(idbuf, raw, 128)
        h = ctypes.c_void_p()
        t0 = time.perf_counter()
        rc = self._rt("edl_rccl_init", idbuf.raw, world, rank, self.device.index or 0, ctypes.byref(self._abort_flag),
                      float(timeout_s), ctypes.byref(h))
        if rc != 0:
            raise RcclError(f"RCCL communicator init (rank {rank}/{world}) failed: {_err(rc)}")
        self._h = h
        self.init_s = time.perf_counter() - t0
        self.stream = torch.cuda.Stream(self.device, priority=-1)

    # -- lifecycle -----------------------------------------------------------
    def abort(self) -> None:
        """Callable from any thread: abandons a pending init, aborts in-flight collectives."""
        self._abort_flag.value = 1
        self._aborted = True
        if self._h is not None:
            self._rt("edl_rccl_abort", self._h)

    def destroy(self) -> None:
        if self._h is not None and not self._aborted:
            self._rt("edl_rccl_destroy", self._h)
        self._h = None

    def async_error(self) -> int:
        return 0 if self._h is None else self._rt("edl_rccl_async_error", self._h)

    def shrink(self, exclude: list[int], timeout_s: float = 60.0) -> "RcclComm":
        """New communicator without ``exclude`` ranks (raises if RCCL lacks ncclCommShrink)."""
        arr = (ctypes.c_int * max(1, len(exclude)))(*exclude)
        h = ctypes.c_void_p()
        rc = self._rt("edl_rccl_shrink", self._h, arr, len(exclude), 1, ctypes.byref(self._abort_flag),
                      float(timeout_s), ctypes.byref(h))
        if rc != 0:
            raise RcclError(f"ncclCommShrink failed: {_err(rc)}")
        new = object.__new__(RcclComm)
        new.__dict__.update(self.__dict__)
        new._h, new._abort_flag, new._aborted = h, ctypes.c_int(0), False
        new.rank = self.rank - sum(1 for r in exclude if r < self.rank)
        new.world_size = self.world_size - len(exclude)
        return new

    # -- collectives ---------------------------------------------------------
    def _launch(self, fn: str, *args, tensors=()):
        if self._aborted or self._h is None:
            raise RcclError("communicator aborted")
        cur = torch.cuda.current_stream(self.device)
        self.stream.wait_stream(cur)
        rc = self._rt(fn, self._h, *args, ctypes.c_void_p(self.stream.cuda_stream))
        if rc != 0:
            raise RcclError(f"{fn} failed: {_err(rc)}")
        for t in tensors:
            t.record_stream(self.stream)
        ev = torch.cuda.Event()
        ev.record(self.stream)
        return _Work(ev, tensors)

    def all_reduce_async(self, t: torch.Tensor, op=dist.ReduceOp.SUM):
        return self._launch("edl_rccl_all_reduce", ctypes.c_void_p(t.data_ptr()), ctypes.c_void_p(t.data_ptr()),
                            t.numel(), _DT[t.dtype], _OP[op], tensors=(t,))

    def broadcast_async(self, t: torch.Tensor, src: int):
        return self._launch("edl_rccl_broadcast", ctypes.c_void_p(t.data_ptr()), ctypes.c_void_p(t.data_ptr()),
                            t.numel(), _DT[t.dtype], src, tensors=(t,))

    def reduce_scatter_async(self, out: torch.Tensor, inp: torch.Tensor, op=dist.ReduceOp.SUM):
        return self._launch("edl_rccl_reduce_scatter", ctypes.c_void_p(inp.data_ptr()),
                            ctypes.c_void_p(out.data_ptr()), out.numel(), _DT[out.dtype], _OP[op],
                            tensors=(out, inp))

    def all_gather_async(self, out: torch.Tensor, inp: torch.Tensor):
        return self._launch("edl_rccl_all_gather", ctypes.c_void_p(inp.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                            inp.numel(), _DT[inp.dtype], tensors=(out, inp))

    def sendrecv_async(self, ops: list[tuple[str, torch.Tensor, int]]):
        """Grouped point-to-point: ops = [("send"|"recv", tensor, peer), ...] (one dtype)."""
        n = len(ops)
        is_send = (ctypes.c_int * n)(*[1 if o == "send" else 0 for o, _, _ in ops])
        bufs = (ctypes.c_void_p * n)(*[t.data_ptr() for _, t, _ in ops])
        counts = (ctypes.c_size_t * n)(*[t.numel() for _, t, _ in ops])
        peers = (ctypes.c_int * n)(*[p for _, _, p in ops])
        return self._launch("edl_rccl_sendrecv", n, is_send, bufs, counts, peers, _DT[ops[0][1].dtype],
                            tensors=tuple(t for _, t, _ in ops))
