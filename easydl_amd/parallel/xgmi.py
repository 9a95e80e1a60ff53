"""Custom xGMI collective engine (csrc/kernels/xgmi.hip + csrc/runtime/xgmi.cpp;
SURVEY.md N3): IPC-mapped peer memory on one node, every wait bounded by an
abort word and a deadline.

* **staged** collectives (any tensor): one-shot all-reduce for small messages,
  two-shot (direct reduce-scatter + all-gather over all 7 links) for large
  ones, MAX all-reduce, all-gather, reduce-scatter — through a per-rank
  workspace with two buffers by round parity;
* **in-place** all-reduce on *registered* buffers: ElasticDDP registers the
  flat gradient buffers once per epoch (:meth:`register`), after which every
  bucket all-reduce is ONE launch that reads the peers' gradient slices where
  they are (no staging copy, no workspace-size split).

Usage (one object per rank and epoch; every rank issues the same calls)::

    x = XgmiComm(store, "edl/job/e3/xgmi", rank, world, device)
    x.register(flat_grad)     # optional, collective
    x.all_reduce(t)           # in place, on the current stream
    x.abort()                 # watchdog thread: spinning kernels give up
    x.status_detail()         # which round / phase / workgroup / peer gave up

Ranks that share one GPU (single-GPU drills) are detected through the store
(device UUIDs) and the grid is capped so every rank's workgroups can be
resident together — the per-workgroup barrier needs workgroup b of every rank
running at once.

Limits: <= 8 ranks (one node), fp32 / bf16, sizes a multiple of 16 bytes.
"""
from __future__ import annotations

import ctypes
import os

import torch

from easydl_amd import _native

STATUS_FIELDS = ("gave_up", "round", "phase", "block", "peer", "peer_flag", "waited_ms", "reason")
REASONS = {0: "", 1: "abort", 2: "deadline"}


class XgmiError(RuntimeError):
    pass


class XgmiAborted(XgmiError):
    """The engine was aborted (abort word set: a peer of this epoch is gone)."""


class _Work:
    def __init__(self, event: torch.cuda.Event, keep):
        self._event, self._keep = event, keep

    def wait(self, *a, **k):
        torch.cuda.current_stream().wait_event(self._event)
        self._keep = None
        return True

    def is_completed(self):
        return self._event.query()


class _Registered:
    """One registered tensor: its base pointer as mapped on every rank."""

    def __init__(self, tensor: torch.Tensor, peers: list[int], opened: list[int]):
        self.tensor = tensor
        self.lo = tensor.data_ptr()
        self.hi = self.lo + tensor.numel() * tensor.element_size()
        self.peers = peers          # rank q's copy of tensor[0], valid in this process
        self.opened = opened        # (peer, handle) keys of the IPC mappings it holds a reference on


class XgmiComm:
    # bytes: below this latency dominates -> one-shot.  The epoch's probe (and the Brain's
    # runtime plan) overwrite the per-instance switch sizes with measured crossovers
    # (parallel/comm_policy.py): ``oneshot_max`` against the in-place two-shot on
    # registered buffers, ``oneshot_max_staged`` against the staged two-shot
    ONESHOT_MAX = 512 << 10
    DEFAULT_WS = 128 << 20       # per parity: one 128 MiB bucket / TP message per launch
    # hipIpcOpenMemHandle of a caching-allocator segment of >= 2 GiB never returns on the
    # box (2040 MiB opens in ms, 2056 MiB hangs: profiles/r03_ipc_size_probe*.txt), so a
    # tensor whose SEGMENT is that large on any rank is not registered (its all-reduces
    # take the staged path, its state transfer the staged pull)
    REGISTER_MAX = int(os.environ.get("EDL_XGMI_REGISTER_MAX_MB", 2040)) << 20

    _FAIL = b"FAIL:"

    def _fail(self, store, prefix: str, rank: int, msg: str) -> None:
        """This rank cannot take part: publish a failure marker in place of its handles (so every
        peer gives up the engine at once, ``__init__``), then raise."""
        try:
            store.set(f"{prefix}/ipc/{rank}", self._FAIL + msg.encode()[:200])
        except Exception:  # noqa: BLE001 - the raise below still ends this rank's attempt
            pass
        raise XgmiError(msg)

    def __init__(self, store, prefix: str, rank: int, world: int, device, ws_bytes: int | None = None,
                 timeout_s: float = 60.0):
        self.rank, self.world_size = rank, world
        self.device = torch.device(device)
        self.timeout_s = timeout_s
        self._store, self._prefix = store, prefix
        self._rt, self._k = _native.runtime(), _native.kernels()
        if world > self._k("edl_xgmi_max_ranks"):
            raise XgmiError(f"xGMI engine supports at most {self._k('edl_xgmi_max_ranks')} ranks")
        ws_bytes = int(ws_bytes or int(os.environ.get("EDL_XGMI_WS_MB", 0)) << 20 or self.DEFAULT_WS)
        h = ctypes.c_void_p()
        rc = self._rt("edl_xgmi_ws_create", self.device.index or 0, ws_bytes, ctypes.byref(h))
        if rc != 0:
            self._fail(store, prefix, rank, f"workspace allocation failed: hipError {rc}")
        self._ws = h
        self.ws_bytes = self._rt("edl_xgmi_ws_bytes", h)
        mine = ctypes.create_string_buffer(128)
        rc = self._rt("edl_xgmi_ws_handles", h, mine)
        # fault injection (tests): these ranks fail their export as hipIpcGetMemHandle once did on a
        # world-8 drill's re-formed epoch (profiles/r06_world8_engine_fail.md)
        if str(rank) in os.environ.get("EDL_XGMI_FAIL_EXPORT", "").split(","):
            rc = 1
        if rc != 0:
            self._rt("edl_xgmi_ws_destroy", h)
            self._ws = None
            self._fail(store, prefix, rank, f"hipIpcGetMemHandle failed: hipError {rc}")
        # device identity travels with the handles: ranks on the SAME GPU are counted
        uuid = str(torch.cuda.get_device_properties(self.device).uuid).encode()[:64].ljust(64, b" ")
        store.set(f"{prefix}/ipc/{rank}", mine.raw + uuid)
        entries = [mine.raw + uuid if p == rank else store.get(f"{prefix}/ipc/{p}") for p in range(world)]
        failed = [p for p, e in enumerate(entries) if e.startswith(self._FAIL)]
        if failed:
            # a peer could not export its workspace: nobody builds the engine this epoch (the peers
            # learn it at once from its marker instead of waiting out the store timeout for a key
            # that never comes, which left them 300 s behind the rank that had fallen back)
            self._rt("edl_xgmi_ws_destroy", h)
            self._ws = None
            raise XgmiError(f"peer rank(s) {failed} could not export their workspace: "
                            f"{entries[failed[0]][len(self._FAIL):].decode(errors='replace')[:120]}")
        allh = b"".join(e[:128] for e in entries)
        # the most ranks any one GPU carries (every rank sees the same records): the grid cap
        # below must be identical on every rank, since workgroup b meets workgroup b of each peer
        per_uuid: dict[bytes, int] = {}
        for e in entries:
            per_uuid[e[128:]] = per_uuid.get(e[128:], 0) + 1
        self.ranks_per_device = max(per_uuid.values())
        rc = self._rt("edl_xgmi_ws_open", h, world, rank, allh)
        if rc != 0:
            raise XgmiError(f"hipIpcOpenMemHandle failed: hipError {rc}")
        self._data = (ctypes.c_void_p * (2 * world))()
        self._flags = (ctypes.c_void_p * world)()
        self._rt("edl_xgmi_ws_ptrs", h, self._data, self._flags)
        self._abort_dev = self._rt("edl_xgmi_ws_abort_dev", h)
        self._status_dev = self._rt("edl_xgmi_ws_status_dev", h)
        self.round = 0
        # Workgroup b of every rank meets workgroup b of every peer (per-workgroup barrier),
        # so all ranks' grids must be resident together.  One rank per GPU: 256 workgroups
        # of 512 threads use at most half the chip.  Ranks SHARING a GPU split the chip and
        # also leave room for the compute kernels running beside the engine.
        hw = min(self._k("edl_xgmi_max_blocks"), 256)
        cap = int(os.environ.get("EDL_XGMI_MAX_BLOCKS", hw))
        if self.ranks_per_device > 1:
            cap = min(cap, max(4, 128 // self.ranks_per_device))
        self.blocks = max(1, min(hw, cap))
        # bucket all-reduces overlap backward: a bounded share of CUs (Brain-tunable)
        self.async_blocks = max(1, min(self.blocks, int(os.environ.get("EDL_XGMI_ASYNC_BLOCKS", 64))))
        self.oneshot_max = self.oneshot_max_staged = self.ONESHOT_MAX
        self._aborted = False
        self._registered: list[_Registered] = []
        self._opened: dict[tuple[int, bytes], list] = {}   # (peer, handle) -> [mapped base, refcount]
        self._reg_seq = 0
        self.stream = torch.cuda.Stream(self.device, priority=-1)

    # -- health -----------------------------------------------------------------
    def abort(self) -> None:
        """From any thread: every spinning workgroup of every in-flight call exits."""
        self._aborted = True
        if self._ws is not None:
            self._rt("edl_xgmi_ws_set_abort", self._ws, 1)

    @property
    def aborted(self) -> bool:
        return self._aborted

    def status(self) -> int:
        """0 = every barrier so far completed; 1 = one gave up (abort / deadline).
        Valid once the caller has synchronised with the collectives it asks about."""
        return self._rt("edl_xgmi_ws_status", self._ws)

    def status_detail(self) -> dict:
        """The give-up record: round, phase, workgroup, missing peer, its last flag, waited ms, reason."""
        out = (ctypes.c_int * 8)()
        self._rt("edl_xgmi_ws_status_detail", self._ws, out)
        d = dict(zip(STATUS_FIELDS, list(out)))
        d["reason"] = REASONS.get(d["reason"], str(d["reason"]))
        return d

    # -- registered buffers ------------------------------------------------------
    def registrable(self, t: torch.Tensor) -> bool:
        """Small enough that mapping it can work (the segment check happens in register)."""
        return t.numel() * t.element_size() <= self.REGISTER_MAX

    def register(self, t: torch.Tensor, any_dtype: bool = False) -> "_Registered":
        """Map ``t`` (this rank's copy of a buffer every rank registers in the same
        order, e.g. a flat gradient group) on every peer.  Collective.  Later
        all-reduces of any 16-byte-aligned slice of it run in place."""
        if not (self.pullable(t) if any_dtype else self.supports(t)):
            raise XgmiError("register: contiguous fp32 / bf16 tensor of 16-byte multiple expected")
        if not self.registrable(t):
            raise XgmiError(f"register: {t.numel() * t.element_size() >> 20} MiB exceeds the IPC mapping limit")
        self._reg_seq += 1
        h = ctypes.create_string_buffer(64)
        off, seg = ctypes.c_uint64(), ctypes.c_uint64()
        rc = self._rt("edl_xgmi_buf_handle", t.data_ptr(), h, ctypes.byref(off), ctypes.byref(seg))
        if rc != 0:   # (still publish, so the peers do not wait forever for this record)
            h, seg = ctypes.create_string_buffer(64), ctypes.c_uint64(1 << 62)
        key = f"{self._prefix}/reg/{self._reg_seq}"
        mine = h.raw + int(off.value).to_bytes(8, "little") + int(seg.value).to_bytes(8, "little")
        self._store.set(f"{key}/{self.rank}", mine)
        entries = [mine if p == self.rank else self._store.get(f"{key}/{p}") for p in range(self.world_size)]
        biggest = max(int.from_bytes(e[72:80], "little") for e in entries)
        if biggest > self.REGISTER_MAX:
            # every rank sees the same records, so every rank gives up on this tensor
            raise XgmiError(f"register: a {biggest >> 20} MiB segment exceeds the IPC mapping limit")
        peers, opened = [], []
        for p in range(self.world_size):
            if p == self.rank:
                peers.append(t.data_ptr())
                continue
            e = entries[p]
            hp, op = e[:64], int.from_bytes(e[64:72], "little")
            ent = self._opened.get((p, hp))
            if ent is None:   # segments shared by several registrations are mapped once
                ptr = ctypes.c_void_p()
                rc = self._rt("edl_xgmi_buf_open", self.device.index or 0, hp, ctypes.byref(ptr))
                if rc != 0:
                    raise XgmiError(f"register: hipIpcOpenMemHandle failed: hipError {rc}")
                ent = self._opened[(p, hp)] = [ptr.value, 0]
            ent[1] += 1
            opened.append((p, hp))
            peers.append(ent[0] + op)
        r = _Registered(t, peers, opened)
        self._registered.append(r)
        return r

    def unregister(self, r: "_Registered") -> None:
        """Drop a registration (after this rank's stream has passed every kernel using it)."""
        if r in self._registered:
            self._registered.remove(r)
        for key in r.opened:
            ent = self._opened.get(key)
            if ent is None:
                continue
            ent[1] -= 1
            if ent[1] == 0:
                self._rt("edl_xgmi_buf_close", self.device.index or 0, ent[0])
                del self._opened[key]
        r.opened = []

    def pull(self, tensors, holders) -> None:
        """State transfer: every rank not in ``holders`` copies each tensor from the
        holders (slice k from holder k, all holders at once over distinct links);
        holders only take part in the entry / exit barriers.  Collective; runs on
        the caller's stream, returns after the launches (sync the stream, then
        check :meth:`status`)."""
        holders = sorted(set(int(h) for h in holders))
        if not holders or holders[0] < 0 or holders[-1] >= self.world_size:
            raise XgmiError(f"pull: bad holder set {holders}")
        mask = sum(1 << h for h in holders)
        stream = torch.cuda.current_stream(self.device)
        nb = int(max(len(holders), min(self.blocks, 256) // len(holders) * len(holders)))
        for t in tensors:
            if not self.pullable(t):
                raise XgmiError("pull: contiguous tensors of 16-byte multiples expected")
        small, regs, big = [], [], []
        for t in tensors:   # registration is collective and agreed: every rank splits alike
            try:
                regs.append(self.register(t, any_dtype=True) if self.registrable(t) else None)
            except XgmiError:
                regs.append(None)
            (small if regs[-1] is not None else big).append(t)
        regs = [r for r in regs if r is not None]
        # too large to map: windows staged through the holders' workspaces
        nh = len(holders)
        win = (self.ws_bytes // 16) * 16 * nh
        for t in big:
            nbytes = t.numel() * t.element_size()
            for off in range(0, nbytes, win):
                w = min(win, nbytes - off)
                self.round += 1
                rc = self._k("edl_xgmi_pull_staged", self._data, self._flags, self.world_size, self.rank,
                             t.data_ptr(), t.data_ptr(), off, w, mask, self.round, nb, self._abort_dev,
                             float(self.timeout_s), self._status_dev, stream.cuda_stream)
                if rc != 0:
                    raise XgmiError(f"launch failed: hipError {rc}")
        try:
            for t, r in zip(small, regs):
                bufs = (ctypes.c_void_p * self.world_size)(*r.peers)
                self.round += 1
                rc = self._k("edl_xgmi_pull", bufs, self._flags, self.world_size, self.rank,
                             t.numel() * t.element_size(), mask, self.round, nb, self._abort_dev,
                             float(self.timeout_s), self._status_dev, stream.cuda_stream)
                if rc != 0:
                    raise XgmiError(f"launch failed: hipError {rc}")
        finally:
            stream.synchronize()
            for r in regs:
                self.unregister(r)

    def _find_registered(self, t: torch.Tensor):
        lo = t.data_ptr()
        hi = lo + t.numel() * t.element_size()
        for r in self._registered:
            if r.lo <= lo and hi <= r.hi and r.tensor.dtype == t.dtype:
                return r, lo - r.lo
        return None, 0

    # -- launches ----------------------------------------------------------------
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
        return self._serialized(self._all_reduce, t, algo, self.blocks)

    def _dtype_code(self, t) -> int:
        return 0 if t.dtype == torch.float32 else 1

    def _all_reduce(self, t: torch.Tensor, algo: str | None = None, max_blocks: int | None = None) -> torch.Tensor:
        if self._aborted:
            raise XgmiAborted("aborted")
        if not self.supports(t):
            raise XgmiError("xGMI all-reduce takes contiguous fp32 / bf16 tensors of 16-byte multiples")
        max_blocks = max_blocks or self.blocks
        flat = t.view(-1)
        es = flat.element_size()
        stream = torch.cuda.current_stream(self.device).cuda_stream
        nbytes_all = flat.numel() * es
        reg, off = self._find_registered(t) if algo in (None, "inplace") else (None, 0)
        if reg is not None and (nbytes_all > self.oneshot_max or algo == "inplace"):
            bufs = (ctypes.c_void_p * self.world_size)(*[p + off for p in reg.peers])
            nvec = nbytes_all // 16
            blocks = int(max(1, min(max_blocks, -(-nvec // (self.world_size * 1024)))))
            self.round += 1
            rc = self._k("edl_xgmi_allreduce_inplace", bufs, self._flags, self.world_size, self.rank, nbytes_all,
                         self._dtype_code(t), self.round, blocks, self._abort_dev, float(self.timeout_s),
                         self._status_dev, stream)
            if rc != 0:
                raise XgmiError(f"launch failed: hipError {rc}")
            return t
        piece = (self.ws_bytes // 16) * 16 // es
        os_max = self.oneshot_max if reg is not None else self.oneshot_max_staged
        for lo in range(0, flat.numel(), piece):
            part = flat[lo:lo + piece]
            nbytes = part.numel() * es
            a = (0 if nbytes <= os_max else 1) if algo in (None, "inplace") else \
                (0 if algo == "oneshot" else 1)
            nvec = nbytes // 16
            per_block = 2048 if a == 0 else 4096  # 16-byte vectors per workgroup before adding workgroups
            blocks = int(max(1, min(max_blocks, -(-nvec // per_block))))
            self.round += 1
            rc = self._k("edl_xgmi_allreduce", self._data, self._flags, self.world_size, self.rank,
                         part.data_ptr(), part.data_ptr(), nbytes, self._dtype_code(t), a,
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
            raise XgmiAborted("aborted")
        for t in ts:
            if not self.supports(t):
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

    def barrier(self) -> None:
        """Device-side barrier of every rank's engine stream (flags only)."""
        def run():
            self.round += 1
            rc = self._k("edl_xgmi_barrier", self._flags, self.world_size, self.rank, self.round, self._abort_dev,
                         float(self.timeout_s), self._status_dev, torch.cuda.current_stream(self.device).cuda_stream)
            if rc != 0:
                raise XgmiError(f"launch failed: hipError {rc}")
        self._serialized(run)

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

    def all_reduce_async(self, t: torch.Tensor, algo: str | None = None) -> "_Work":
        """In-place SUM on the engine's own high-priority stream, ordered after the
        caller's stream; ``wait()`` orders the caller's stream after it (the
        ``ProcessGroupNCCL`` work contract ElasticDDP overlaps with backward).
        Uses at most ``async_blocks`` workgroups so backward keeps most CUs.
        ``algo`` pins a form (the policy probe times each one in this configuration)."""
        self.stream.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self.stream):
            self._all_reduce(t, algo, self.async_blocks)
        t.record_stream(self.stream)
        ev = torch.cuda.Event()
        ev.record(self.stream)
        return _Work(ev, t)

    @staticmethod
    def pullable(t: torch.Tensor) -> bool:
        """Byte copies (state transfer) take any dtype."""
        return (t.is_cuda and t.is_contiguous() and (t.numel() * t.element_size()) % 16 == 0
                and t.data_ptr() % 16 == 0 and t.numel() > 0)

    @staticmethod
    def supports(t: torch.Tensor) -> bool:
        return (t.is_cuda and t.dtype in (torch.float32, torch.bfloat16) and t.is_contiguous()
                and (t.numel() * t.element_size()) % 16 == 0 and t.data_ptr() % 16 == 0)

    def close_after_abort(self) -> None:
        """Release an aborted engine: its spinning workgroups leave on the abort word (bounded
        by the deadline in any case), so only this engine's stream is drained; then every IPC
        mapping is closed -- including those of a dead peer's buffers, which would otherwise
        keep that peer's HBM allocated on its GPU -- and the workspace freed.  May run on a
        background thread (hipStreamSynchronize and the unmaps are thread-safe)."""
        if self._ws is None:
            return
        self.abort()
        self.stream.synchronize()
        for base, _ in self._opened.values():
            self._rt("edl_xgmi_buf_close", self.device.index or 0, base)
        self._registered, self._opened = [], {}
        self._rt("edl_xgmi_ws_destroy", self._ws)
        self._ws = None

    def close(self) -> None:
        """Unmap registered buffers and free the workspace.  Called after a committed
        step, when every rank has synced its streams, so no engine kernel is in flight
        anywhere.  Only this engine's stream is drained: a device-wide sync would also
        wait for an in-flight snapshot copy (up to ~0.5 s at a world change,
        profiles/r02_ttr_rejoin_*)."""
        if self._ws is not None:
            torch.cuda.current_stream(self.device).synchronize()
            self.stream.synchronize()
            for base, _ in self._opened.values():
                self._rt("edl_xgmi_buf_close", self.device.index or 0, base)
            self._registered, self._opened = [], {}
            self._rt("edl_xgmi_ws_destroy", self._ws)
            self._ws = None
