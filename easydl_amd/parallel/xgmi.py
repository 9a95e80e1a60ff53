"""Custom xGMI all-reduce (csrc/kernels/xgmi.hip + csrc/runtime/xgmi.cpp;
SURVEY.md N3): IPC-mapped peer buffers on one node, one-shot for small
messages, two-shot (direct reduce-scatter + all-gather over all 7 links) for
large ones, every wait bounded by an abort word and a deadline.

Usage (one object per rank and epoch; every rank issues the same calls)::

    x = XgmiComm(store, "edl/job/e3/xgmi", rank, world, device)
    x.all_reduce(t)           # in place, on the current stream
    x.abort()                 # watchdog thread: spinning kernels give up

Also ``all_reduce_max``, ``all_gather`` and ``reduce_scatter`` (the TP / SP
collectives; ``Communicator(data_backend="xgmi")`` routes them here).

Limits: <= 8 ranks (one node), fp32 / bf16, sizes a multiple of 16 bytes
(tensors are processed in workspace-sized pieces).
"""
from __future__ import annotations

import ctypes
import os

import torch

from easydl_amd import _native


class XgmiError(RuntimeError):
    pass


class _Work:
    def __init__(self, event: torch.cuda.Event, keep):
        self._event, self._keep = event, keep

    def wait(self, *a, **k):
        torch.cuda.current_stream().wait_event(self._event)
        self._keep = None
        return True

    def is_completed(self):
        return self._event.query()


class XgmiComm:
    ONESHOT_MAX = 512 << 10      # bytes: below this latency dominates -> one-shot

    def __init__(self, store, prefix: str, rank: int, world: int, device, ws_bytes: int = 64 << 20,
                 timeout_s: float = 60.0):
        self.rank, self.world_size = rank, world
        self.device = torch.device(device)
        self.timeout_s = timeout_s
        self._rt, self._k = _native.runtime(), _native.kernels()
        if world > self._k("edl_xgmi_max_ranks"):
            raise XgmiError(f"xGMI all-reduce supports at most {self._k('edl_xgmi_max_ranks')} ranks")
        h = ctypes.c_void_p()
        rc = self._rt("edl_xgmi_ws_create", self.device.index or 0, ws_bytes, ctypes.byref(h))
        if rc != 0:
            raise XgmiError(f"workspace allocation failed: hipError {rc}")
        self._ws = h
        self.ws_bytes = self._rt("edl_xgmi_ws_bytes", h)
        mine = ctypes.create_string_buffer(128)
        rc = self._rt("edl_xgmi_ws_handles", h, mine)
        if rc != 0:
            raise XgmiError(f"hipIpcGetMemHandle failed: hipError {rc}")
        store.set(f"{prefix}/ipc/{rank}", mine.raw)
        allh = b"".join(mine.raw if p == rank else store.get(f"{prefix}/ipc/{p}") for p in range(world))
        rc = self._rt("edl_xgmi_ws_open", h, world, rank, allh)
        if rc != 0:
            raise XgmiError(f"hipIpcOpenMemHandle failed: hipError {rc}")
        self._data = (ctypes.c_void_p * (2 * world))()
        self._flags = (ctypes.c_void_p * world)()
        self._rt("edl_xgmi_ws_ptrs", h, self._data, self._flags)
        self._abort_dev = self._rt("edl_xgmi_ws_abort_dev", h)
        self._status_dev = self._rt("edl_xgmi_ws_status_dev", h)
        self.round = 0
        # Workgroup b of every rank meets workgroup b of every peer (per-block barrier), so
        # all ranks' workgroups must be resident together.  One rank per GPU: always true.
        # Ranks SHARING a GPU (EDL_XGMI_MAX_BLOCKS set by the shared-GPU drills): 4 ranks x
        # 256 x 512 threads would fill every thread slot of the chip and a late rank's
        # workgroups could never be dispatched, so the grid is capped.
        cap = int(os.environ.get("EDL_XGMI_MAX_BLOCKS", 256))
        self.blocks = max(1, min(self._k("edl_xgmi_max_blocks"), 256, cap))
        self._aborted = False
        self.stream = torch.cuda.Stream(self.device, priority=-1)

    def abort(self) -> None:
        """From any thread: every spinning workgroup of every in-flight call exits."""
        self._aborted = True
        if self._ws is not None:
            self._rt("edl_xgmi_ws_set_abort", self._ws, 1)

    @property
    def aborted(self) -> bool:
        return self._aborted

    def status(self) -> int:
        """0 = every barrier so far completed; 1 = one gave up (abort / deadline). Synchronising."""
        return self._rt("edl_xgmi_ws_status", self._ws)

    # Every kernel of this comm runs on ONE stream (self.stream).  The workspace's
    # round-parity buffers are only safe if a rank's rounds execute one after
    # another: a sync collective issued while async bucket all-reduces are still
    # pending must queue behind them, never run beside them.
    def _serialized(self, fn, *args):
        caller = torch.cuda.current_stream(self.device)
        if caller == self.stream:
            return fn(*args)
        self.stream.wait_stream(caller)
        with torch.cuda.stream(self.stream):
            out = fn(*args)
        caller.wait_stream(self.stream)
        return out

    def all_reduce(self, t: torch.Tensor, algo: str | None = None) -> torch.Tensor:
        return self._serialized(self._all_reduce, t, algo)

    def _all_reduce(self, t: torch.Tensor, algo: str | None = None) -> torch.Tensor:
        if self._aborted:
            raise XgmiError("aborted")
        if t.dtype not in (torch.float32, torch.bfloat16) or not t.is_contiguous():
            raise XgmiError("xGMI all-reduce takes contiguous fp32 / bf16 tensors")
        flat = t.view(-1)
        es = flat.element_size()
        if (flat.numel() * es) % 16:
            raise XgmiError("size must be a multiple of 16 bytes")
        piece = (self.ws_bytes // 16) * 16 // es
        stream = torch.cuda.current_stream(self.device).cuda_stream
        for lo in range(0, flat.numel(), piece):
            part = flat[lo:lo + piece]
            nbytes = part.numel() * es
            a = (0 if nbytes <= self.ONESHOT_MAX else 1) if algo is None else (0 if algo == "oneshot" else 1)
            nvec = nbytes // 16
            per_block = 2048 if a == 0 else 4096  # 16-byte vectors per workgroup before adding workgroups
            blocks = int(max(1, min(self.blocks, -(-nvec // per_block))))
            self.round += 1
            rc = self._k("edl_xgmi_allreduce", self._data, self._flags, self.world_size, self.rank,
                         part.data_ptr(), part.data_ptr(), nbytes, 0 if t.dtype == torch.float32 else 1, a,
                         self.round, blocks, self._abort_dev, float(self.timeout_s), self._status_dev, stream)
            if rc != 0:
                raise XgmiError(f"launch failed: hipError {rc}")
        return t

    # -- TP / SP collectives (one-shot MAX, all-gather, reduce-scatter) --------------
    def _launch(self, kind: int, inp_ptr: int, out_ptr: int, nvec: int, stride: int, dtype, nblocks_hint: int):
        blocks = int(max(1, min(self.blocks, -(-nblocks_hint // 2048))))
        self.round += 1
        stream = torch.cuda.current_stream(self.device).cuda_stream
        rc = self._k("edl_xgmi_collective", self._data, self._flags, self.world_size, self.rank, inp_ptr, out_ptr,
                     nvec, stride, 0 if dtype == torch.float32 else 1, kind, self.round, blocks, self._abort_dev,
                     float(self.timeout_s), self._status_dev, stream)
        if rc != 0:
            raise XgmiError(f"launch failed: hipError {rc}")

    def _check(self, *ts):
        if self._aborted:
            raise XgmiError("aborted")
        for t in ts:
            if t.dtype not in (torch.float32, torch.bfloat16) or not t.is_contiguous() or \
                    (t.numel() * t.element_size()) % 16:
                raise XgmiError("xGMI collectives take contiguous fp32 / bf16 tensors of 16-byte multiples")

    def all_reduce_max(self, t: torch.Tensor) -> torch.Tensor:
        """In-place element-wise MAX over ranks (one-shot)."""
        return self._serialized(self._all_reduce_max, t)

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor) -> torch.Tensor:
        """out = concat over ranks of inp (rank-major), read directly from every peer."""
        return self._serialized(self._all_gather, out, inp)

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor) -> torch.Tensor:
        """out = SUM over ranks of this rank's slice of inp (inp = world_size slices, rank-major)."""
        return self._serialized(self._reduce_scatter, out, inp)

    def _all_reduce_max(self, t: torch.Tensor) -> torch.Tensor:
        self._check(t)
        flat = t.view(-1)
        es = flat.element_size()
        piece = self.ws_bytes // es
        for lo in range(0, flat.numel(), piece):
            part = flat[lo:lo + piece]
            nvec = part.numel() * es // 16
            self._launch(0, part.data_ptr(), part.data_ptr(), nvec, 0, t.dtype, nvec)
        return t

    def _all_gather(self, out: torch.Tensor, inp: torch.Tensor) -> torch.Tensor:
        self._check(out, inp)
        if out.dtype != inp.dtype or out.numel() != inp.numel() * self.world_size:
            raise XgmiError("all_gather: out must hold world_size x inp")
        es = inp.element_size()
        n = inp.numel()
        stride = n * es // 16
        piece = (self.ws_bytes // 16) * 16 // es
        src, dst = inp.view(-1), out.view(-1)
        for lo in range(0, n, piece):
            m = min(piece, n - lo)
            self._launch(1, src[lo:].data_ptr(), dst[lo:].data_ptr(), m * es // 16, stride, inp.dtype, m * es // 16)
        return out

    def _reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor) -> torch.Tensor:
        self._check(out, inp)
        if out.dtype != inp.dtype or inp.numel() != out.numel() * self.world_size:
            raise XgmiError("reduce_scatter: inp must hold world_size x out")
        es = out.element_size()
        n = out.numel()
        stride = n * es // 16
        piece = (self.ws_bytes // self.world_size // 16) * 16 // es   # all slices are staged
        src, dst = inp.view(-1), out.view(-1)
        for lo in range(0, n, piece):
            m = min(piece, n - lo)
            self._launch(2, src[lo:].data_ptr(), dst[lo:].data_ptr(), m * es // 16, stride, out.dtype, m * es // 16)
        return out

    def all_reduce_async(self, t: torch.Tensor) -> "_Work":
        """In-place SUM on the engine's own high-priority stream, ordered after the
        caller's stream; ``wait()`` orders the caller's stream after it (the
        ``ProcessGroupNCCL`` work contract ElasticDDP overlaps with backward)."""
        self.stream.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self.stream):
            self._all_reduce(t)
        t.record_stream(self.stream)
        ev = torch.cuda.Event()
        ev.record(self.stream)
        return _Work(ev, t)

    @staticmethod
    def supports(t: torch.Tensor) -> bool:
        return (t.is_cuda and t.dtype in (torch.float32, torch.bfloat16) and t.is_contiguous()
                and (t.numel() * t.element_size()) % 16 == 0)

    def close(self) -> None:
        """Free the workspace.  Called after a committed step, when every rank has synced its
        streams, so no engine kernel is in flight anywhere.  Only this engine's stream is
        drained: a device-wide sync would also wait for an in-flight snapshot copy (up to
        ~0.5 s at a world change, profiles/r02_ttr_rejoin_*)."""
        if self._ws is not None:
            torch.cuda.current_stream(self.device).synchronize()
            self.stream.synchronize()
            self._rt("edl_xgmi_ws_destroy", self._ws)
            self._ws = None
