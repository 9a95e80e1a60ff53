"""Parameter server role (reference docs/design/elastic-training-operator.md:39-40,
65-71; README.md:27-35: PS can fail and be recovered, scaled in number and
resources).  SURVEY.md §2.5 P1, CS6.

One PS process owns a shard of the parameters (``partition.assign``) as ONE
flat fp32 buffer with its optimizer state, and serves:

* ``pull``  -> current shard (+ version); in sync mode a pull can wait for a
  minimum version (bounded staleness);
* ``push``  -> gradients of the shard.  **async**: applied on arrival with the
  fused flat AdamW/SGD (HIP kernel when the shard lives on a GPU), version+1;
  **sync**: accumulated until every live worker of the round has pushed
  (membership from the job master's rendezvous), then averaged and applied;
* ``state`` / ``load`` -> full shard + optimizer state (replacement PS restore);
* periodic snapshots of the shard state into operator-owned /dev/shm (the same
  A/B segment store as DDP checkpoints), so a replaced PS resumes where the
  failed one stopped (CS3 vertical scaling / CS4 PS death).

Worker death never stops training in async mode ("some failed nodes do not
interrupt the training", README.md:28): the PS just stops hearing from it.
"""
from __future__ import annotations

import logging
import socket
import zlib
import threading
import time

import torch

from easydl_amd.ops import sparse
from easydl_amd.ops.optim import adamw_flat_, sgd_flat_
from easydl_amd.ps.wire import recv_msg, send_msg

log = logging.getLogger("edl.ps")


class ShardState:
    """A PS shard as flat fp32 buffers: params, grads accumulator, optimizer moments."""

    def __init__(self, tensors: dict[str, torch.Tensor], device="cpu"):
        self.names = list(tensors)
        self.shapes = {n: tuple(t.shape) for n, t in tensors.items()}
        self.offsets = {}
        off = 0
        for n in self.names:
            self.offsets[n] = off
            off += (tensors[n].numel() + 3) // 4 * 4
        self.numel = max(4, off)
        self.device = torch.device(device)
        self.w = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
        for n, t in tensors.items():
            self.view(self.w, n).copy_(t.float())
        self.g = torch.zeros_like(self.w)
        self.m = torch.zeros_like(self.w)
        self.v = torch.zeros_like(self.w)

    def view(self, buf, name):
        o = self.offsets[name]
        k = 1
        for d in self.shapes[name]:
            k *= d
        return buf[o:o + k].view(self.shapes[name])

    def tensors(self, buf=None, names=None) -> dict[str, torch.Tensor]:
        buf = self.w if buf is None else buf
        return {n: self.view(buf, n) for n in (names or self.names)}


class TableShard:
    """This PS's stripe of a row-sparse embedding table (fp32 rows + lazy optimizer state)."""

    def __init__(self, name: str, rows: int, dim: int, init_std: float, index: int, device, seed: int = 1234):
        self.name, self.rows, self.dim = name, max(1, rows), dim
        g = torch.Generator(device="cpu").manual_seed(seed * 1000003 + zlib.crc32(name.encode()) * 31 + index)
        self.w = (torch.randn(self.rows, dim, generator=g) * init_std).to(device)
        self.m = torch.zeros_like(self.w)
        self.v = torch.zeros_like(self.w)
        self.step = 0
        self.pending: list[tuple[torch.Tensor, torch.Tensor]] = []  # sync mode: (ids, grads) of the round

    def apply(self, ids: torch.Tensor, grads: torch.Tensor, *, kind: str, lr: float, betas, eps: float,
              wd: float, scale: float) -> None:
        ids = ids.to(self.w.device)
        grads = grads.to(self.w.device)
        uniq, comp = sparse.segment_sum_rows(ids, grads, self.rows)
        self.step += 1
        sparse.sparse_rows_update(self.w, self.m, self.v, uniq, comp, kind=kind, lr=lr, beta1=betas[0],
                                  beta2=betas[1], eps=eps, weight_decay=wd, step=self.step, scale=scale)


class ParameterServer:
    def __init__(self, index: int, tensors: dict[str, torch.Tensor], *, optimizer: str = "adam", lr: float = 1e-3,
                 betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0, momentum: float = 0.9,
                 mode: str = "async", expected_workers=None, host: str = "127.0.0.1", port: int = 0,
                 device="cpu", snapshot=None, snapshot_every: int = 50, tables: dict[str, dict] | None = None,
                 sparse_optimizer: str | None = None, sparse_lr: float | None = None, seed: int = 1234,
                 snapshot_min_s: float = 0.0):
        self.index = index
        self.state = ShardState(tensors, device)
        # row-sparse embedding stripes (easydl_amd/ps/embedding.py), lazily updated
        self.tables = {n: TableShard(n, t["rows"], t["dim"], t.get("init_std", 0.01), index, device, seed)
                       for n, t in (tables or {}).items()}
        # GPU transport: worker -> two gradient inboxes in this HBM (double buffered) and the
        # completion event of the update that last read each one
        self.inboxes: dict[str, list[torch.Tensor]] = {}
        self._inbox_ev: dict[str, list] = {}
        # ... and, per row-sparse table, two sparse inboxes (local ids, fp32 rows, row count)
        # the worker fills on its GPU; the push flag below orders the PS's reads after those writes
        self.sp_inboxes: dict[str, dict[str, list[tuple]]] = {}
        # push ordering: the worker's stream stores its push sequence number into this flag
        # word after its inbox writes (edl_ps_signal); our stream waits for it (edl_ps_wait,
        # bounded) before the update.  The worker sends push_ipc once its stream has passed the
        # flag store (ps/client.py), so the wait normally returns at once; it guards the order
        self._push_flag: dict[str, torch.Tensor] = {}
        self._push_status: dict[str, torch.Tensor] = {}
        self._apply_ev = None      # completion of the newest update of the shard
        self.sparse_optimizer = sparse_optimizer or ("adam" if optimizer == "adam" else "sgd")
        self.sparse_lr = lr if sparse_lr is None else sparse_lr
        self.optimizer, self.lr, self.betas, self.eps = optimizer, lr, betas, eps
        self.wd, self.momentum = weight_decay, momentum
        self.mode = mode
        self.expected_workers = expected_workers or (lambda: 1)
        self.version = 0
        self.step = 0
        self.lock = threading.Condition()
        self.round_pushers: set[str] = set()
        self.stats = {"pushes": 0, "pulls": 0, "applied": 0, "workers": set()}
        self.snapshot = snapshot
        self.snapshot_every = snapshot_every
        # ... and at least this many seconds apart: a snapshot copies the whole shard state (4 GB
        # for BERT-large) to host DRAM, which on a GPU shared with workers costs copy kernels
        # beside their steps (profiles/r05_ps_per_gpu.md)
        self.snapshot_min_s = snapshot_min_s
        self._last_snap_t = 0.0
        self.push_wait_s = 30.0
        self._srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self._srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self._srv.bind((host, port))
        self._srv.listen(128)
        self.host, self.port = self._srv.getsockname()
        self._stop = threading.Event()
        self._threads = []
        # graceful hand-over (retire): no new requests, in-flight ones finish, final snapshot
        self._retiring = threading.Event()
        self._conns: set = set()
        self._busy = 0
        from easydl_amd.utils.kmix import KernelMixMeter
        self.kmix = KernelMixMeter(self.state.device)   # live kernel mix for the Brain (utils/kmix.py)
        self.events = None           # EventLog of the PS process (run_ps)
        self.on_apply = None         # callback after every update (run_ps: fault injection, first-apply event)

    # -- optimizer -------------------------------------------------------------
    def _fence_snapshot(self) -> None:
        """Order every later write of a snapshotted buffer (dense shard, sparse
        table rows, a restore) after the in-flight D2H copy of the snapshot."""
        st = self.state
        if st.w.is_cuda and hasattr(self.snapshot, "fence"):
            self.snapshot.fence(st.w.device)

    def _apply(self, scale: float, grad: torch.Tensor | None = None) -> None:
        """One optimizer update of the shard from ``grad`` (default: the accumulator)."""
        st = self.state
        g = st.g if grad is None else grad
        self._fence_snapshot()  # never update under an in-flight snapshot copy
        self.step += 1
        if self.optimizer == "adam":
            adamw_flat_(None, st.w, st.m, st.v, g, lr=self.lr, beta1=self.betas[0], beta2=self.betas[1],
                        eps=self.eps, weight_decay=self.wd, step=self.step, scale=scale)
        else:
            sgd_flat_(None, st.w, st.m if self.momentum else None, g, lr=self.lr, momentum=self.momentum,
                      weight_decay=self.wd, scale=scale)
        if grad is None:
            st.g.zero_()
        for t in self.tables.values():
            if t.pending:
                ids = torch.cat([i for i, _ in t.pending])
                grads = torch.cat([g for _, g in t.pending])
                t.pending = []
                self._apply_table(t, ids, grads, scale)
        self.version += 1
        self.stats["applied"] += 1
        if self.on_apply is not None:
            self.on_apply(self)
        if st.w.is_cuda:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(st.device))
            self._apply_ev = ev
        if self.snapshot is not None and self.snapshot_every > 0 and self.version % self.snapshot_every == 0 \
                and time.monotonic() - self._last_snap_t >= self.snapshot_min_s:
            self._last_snap_t = time.monotonic()
            self.snapshot(self)
        self.lock.notify_all()

    def _apply_table(self, t: TableShard, ids, grads, scale: float) -> None:
        t.apply(ids, grads, kind=self.sparse_optimizer, lr=self.sparse_lr, betas=self.betas, eps=self.eps, wd=0.0,
                scale=scale)

    def _apply_sparse(self, grads: dict[str, torch.Tensor], async_mode: bool) -> None:
        for n, t in self.tables.items():
            ids = grads.get(f"sparse/{n}/ids")
            if ids is None or ids.numel() == 0:
                continue
            g = grads[f"sparse/{n}/grad"]
            if async_mode:
                self._apply_table(t, ids, g, 1.0)
            else:
                t.pending.append((ids.to(t.w.device), g.to(t.w.device, torch.float32)))

    def _apply_sparse_inbox(self, worker: str, slot: int, async_mode: bool) -> None:
        """Row-sparse gradients a worker wrote into its sparse inboxes (GPU transport)."""
        for n, t in self.tables.items():
            ids, g, cnt = self.sp_inboxes[worker][n][slot]
            if async_mode:
                t.step += 1
                sparse.sparse_inbox_update(t.w, t.m, t.v, ids, g, cnt, kind=self.sparse_optimizer, lr=self.sparse_lr,
                                           beta1=self.betas[0], beta2=self.betas[1], eps=self.eps, weight_decay=0.0,
                                           step=t.step, scale=1.0)
            else:
                k = int(cnt[0])   # sync rounds wait for every worker anyway: a host read is fine here
                if k:
                    t.pending.append((ids[:k].clone(), g[:k].clone()))

    def _push(self, worker: str, grads: dict[str, torch.Tensor], inbox: torch.Tensor | None = None,
              slot: int = 0, sparse_inbox: bool = False) -> int:
        with self.lock, self.kmix.phase("memory"):   # accumulate + AdamW/Adagrad: HBM-bound
            st = self.state
            # sparse-table rows are updated below, before _apply: they are part of the
            # snapshot too, so the fence must come first
            self._fence_snapshot()
            if sparse_inbox:
                self._apply_sparse_inbox(worker, slot, async_mode=self.mode == "async")
            if inbox is not None and self.mode == "async":
                # GPU transport: the inbox IS the gradient of this update (no accumulate pass);
                # its release is an event, waited for only when the worker wants this slot back
                self._apply_sparse(grads, async_mode=True)
                self.stats["pushes"] += 1
                self.stats["workers"].add(worker)
                self._apply(1.0, grad=inbox)
                self._inbox_ev[worker][slot] = self._apply_ev
                return self.version
            if inbox is not None:
                st.g.add_(inbox)
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream(st.device))
                self._inbox_ev[worker][slot] = ev
            for n, g in grads.items():
                if n.startswith("sparse/"):
                    continue
                st.view(st.g, n).add_(g.to(st.device, torch.float32))
            self._apply_sparse(grads, async_mode=self.mode == "async")
            self.stats["pushes"] += 1
            self.stats["workers"].add(worker)
            if self.mode == "async":
                self._apply(1.0)
                return self.version
            # sync: one contribution per worker per round
            self.round_pushers.add(worker)
            target = self.version + 1
            while self.version < target:
                if len(self.round_pushers) >= max(1, self.expected_workers()) or (
                        self._retiring.is_set() and self.round_pushers):
                    # (retiring: the other workers' pushes go to the successor; close this round)
                    n = len(self.round_pushers)
                    self.round_pushers = set()
                    self._apply(1.0 / n)
                    break
                if not self.lock.wait(timeout=0.05):
                    continue
            return self.version

    # -- serving ---------------------------------------------------------------
    def _serve(self, conn: socket.socket):
        with self.lock:
            self._conns.add(conn)
        try:
            while not self._stop.is_set() and not self._retiring.is_set():
                try:
                    hdr, tensors = recv_msg(conn)
                except (ConnectionError, OSError):
                    return
                with self.lock:
                    if self._retiring.is_set():
                        return     # never started: the client re-sends it to the successor
                    self._busy += 1
                try:
                    self._handle(conn, hdr, tensors)
                finally:
                    with self.lock:
                        self._busy -= 1
                        self.lock.notify_all()
        finally:
            with self.lock:
                self._conns.discard(conn)
            conn.close()

    def _handle(self, conn: socket.socket, hdr: dict, tensors) -> None:
        op = hdr.get("op")
        if op == "pull":
            minv = int(hdr.get("min_version", 0))
            with self.lock:
                t_end = time.monotonic() + float(hdr.get("timeout", 60))
                while self.version < minv and time.monotonic() < t_end:
                    self.lock.wait(timeout=0.05)
                self.stats["pulls"] += 1
                out = {n: t.clone() for n, t in self.state.tensors(names=hdr.get("names")).items()}
                ver = self.version
            send_msg(conn, {"ok": True, "version": ver}, out)
        elif op == "pull_rows":
            t = self.tables[hdr["table"]]
            ids = tensors["ids"].to(t.w.device)
            dt = torch.bfloat16 if hdr.get("bf16") else torch.float32
            with self.lock:
                rows = sparse.embed_gather(t.w, ids, out_dtype=dt)
                ver = self.version
            self.stats["pulls"] += 1
            send_msg(conn, {"ok": True, "version": ver}, {"rows": rows})
        elif op == "ipc_open":
            from easydl_amd.ps.ipc import export_tensor
            st = self.state
            if not st.w.is_cuda:
                send_msg(conn, {"ok": False, "error": "PS shard is not on a GPU"})
                return
            with self.lock:
                wid = hdr.get("worker", "?")
                self._adopt_seen_version(int(hdr.get("seen_version", 0)), wid)
                if wid not in self.inboxes:
                    self.inboxes[wid] = [torch.zeros_like(st.w), torch.zeros_like(st.w)]
                    self._inbox_ev[wid] = [None, None]
                desc = {"w": export_tensor(st.w), "inbox": [export_tensor(x) for x in self.inboxes[wid]],
                        "layout": {n: [st.offsets[n], list(st.shapes[n])] for n in st.names}}
                if wid not in self._push_flag:
                    self._push_flag[wid] = torch.zeros(4, dtype=torch.int32, device=st.device)
                    self._push_status[wid] = torch.zeros(4, dtype=torch.int32, device=st.device)
                else:
                    # a (re)connecting client -- the same worker after a reconnect, or its
                    # replacement -- counts its push sequence from 0 again: restart the flag
                    # in stream order, or every wait for a small seq would pass at once
                    self._push_flag[wid].zero_()
                    self.stats["flag_resets"] = self.stats.get("flag_resets", 0) + 1
                desc["flag"] = export_tensor(self._push_flag[wid])
                cap = int(hdr.get("sparse_cap", 0))
                if self.tables and cap > 0:
                    if wid not in self.sp_inboxes or any(
                            b[0][0].numel() != cap for b in self.sp_inboxes[wid].values()):
                        dev = st.device
                        self.sp_inboxes[wid] = {
                            n: [(torch.zeros(cap, dtype=torch.int64, device=dev),
                                 torch.zeros(cap, t.dim, dtype=torch.float32, device=dev),
                                 torch.zeros(4, dtype=torch.int32, device=dev)) for _ in range(2)]
                            for n, t in self.tables.items()}
                    desc["tables"] = {n: {"w": export_tensor(t.w), "rows": t.rows}
                                      for n, t in self.tables.items()}
                    desc["sparse_inbox"] = {n: [[export_tensor(x) for x in b] for b in bufs]
                                            for n, bufs in self.sp_inboxes[wid].items()}
                    desc["sparse_cap"] = cap
            send_msg(conn, {"ok": True, "ipc": desc, "version": self.version})
        elif op == "pull_ipc":
            minv = int(hdr.get("min_version", 0))
            with self.lock:
                t_end = time.monotonic() + float(hdr.get("timeout", 60))
                while self.version < minv and time.monotonic() < t_end:
                    self.lock.wait(timeout=0.05)
                self.stats["pulls"] += 1
                ver, ev = self.version, self._apply_ev
            if ev is not None:
                ev.synchronize()   # the worker reads the shard next: that version must be written
            send_msg(conn, {"ok": True, "version": ver})
        elif op == "push_ipc":
            wid, slot = hdr["worker"], int(hdr.get("slot", 0))
            if wid not in self.inboxes or wid not in self._push_flag:
                # a worker that mapped a PREVIOUS incarnation of this shard (it died): its
                # gradients are in that PS's inbox, not ours -- it must map this one first
                send_msg(conn, {"ok": False, "error": "remap", "version": self.version})
                return
            if hdr.get("seq") is not None:   # the worker's inbox writes before our reads
                dev = self.state.device
                sparse.ps_wait(self._push_flag[wid], int(hdr["seq"]), self.push_wait_s,
                               self._push_status[wid], torch.cuda.current_stream(dev))
            ver = self._push(wid, tensors, inbox=self.inboxes[wid][slot], slot=slot,
                             sparse_inbox=bool(hdr.get("sparse_ipc")))
            with self.lock:
                other = self._inbox_ev[wid][1 - slot]   # read by the previous push's update
                mine = self._apply_ev if hdr.get("pull") else None
            # outside the lock: other workers' pushes keep flowing meanwhile
            if other is not None:
                other.synchronize()
            if mine is not None:
                mine.synchronize()   # push + pull in one message: the update is written
            if hdr.get("seq") is not None and (other is not None or mine is not None):
                # a bounded wait that gave up (a worker killed mid-push): counted
                stw = self._push_status[wid]
                if int(stw[0]):
                    self.stats["push_wait_timeouts"] = self.stats.get("push_wait_timeouts", 0) + 1
                    log.warning("PS %d: push of %s applied after its ordering wait gave up", self.index,
                                wid)
                    stw.zero_()
            send_msg(conn, {"ok": True, "version": ver})
        elif op == "push":
            ver = self._push(hdr.get("worker", "?"), tensors)
            send_msg(conn, {"ok": True, "version": ver})
        elif op == "state":
            with self.lock:
                out = {f"b{i}": b.clone() for i, b in enumerate(self.state_buffers())}
                meta = {"version": self.version, "step": self.step,
                        "table_steps": [t.step for t in self.tables.values()]}
            send_msg(conn, {"ok": True, **meta}, out)
        elif op == "load":
            with self.lock:
                self._fence_snapshot()
                self.load([tensors[f"b{i}"] for i in range(len(tensors))], hdr["version"], hdr["step"],
                          hdr.get("table_steps"))
            send_msg(conn, {"ok": True})
        elif op == "stats":
            s = dict(self.stats)
            s["workers"] = sorted(s["workers"])
            send_msg(conn, {"ok": True, "version": self.version, "stats": s, "index": self.index})
        elif op == "shutdown":
            send_msg(conn, {"ok": True})
            self._stop.set()
            return
        else:
            send_msg(conn, {"ok": False, "error": f"unknown op {op}"})

    def _adopt_seen_version(self, seen: int, worker: str) -> None:
        """(Lock held.)  A replacement PS restored its newest snapshot (version V_snap), but its
        workers may have seen versions up to V_hwm from the dead PS: the count continues from
        the highest version any worker reports, so versions never go back (sync-mode waits for
        ``min_version`` and bounded staleness rely on that).  ``lost_updates`` = the updates the
        dead PS applied after its last snapshot, as far as the workers saw them."""
        if seen <= self.version:
            return
        base = self.stats.get("restored_version")
        if base is not None:
            self.stats["lost_updates"] = max(self.stats.get("lost_updates", 0), seen - int(base))
        self.stats["version_adopted_from"] = worker
        self.version = seen
        self.lock.notify_all()
        ev = getattr(self, "events", None)
        if ev is not None:
            ev.emit("ps_version_adopted", version=seen, worker=worker, restored_version=base,
                    lost_updates=self.stats.get("lost_updates"))

    def retire(self, timeout_s: float = 60.0) -> int:
        """Graceful hand-over to a successor (vertical resize by replacement, reference
        docs/design/elastic-training-operator.md:99-101): stop accepting connections, cut the
        idle ones (a request already read runs to its reply; one not yet read fails on the
        client, which re-sends it to the successor -- so every acknowledged update is in the
        final snapshot, and none is applied twice), then snapshot the final version and wait
        for the snapshot to be committed.  Returns that version."""
        self._retiring.set()
        try:
            self._srv.close()
        except OSError:
            pass
        with self.lock:
            for c in list(self._conns):
                try:
                    c.shutdown(socket.SHUT_RD)
                except OSError:
                    pass
            self.lock.notify_all()
            t_end = time.monotonic() + timeout_s
            while self._busy and time.monotonic() < t_end:
                self.lock.wait(timeout=0.05)
            if self.snapshot is not None:
                self._fence_snapshot()
                self.snapshot(self)
                wait = getattr(self.snapshot, "wait", None)
                if wait is not None:
                    wait()
            ver = self.version
        self._stop.set()
        return ver

    def state_buffers(self) -> list[torch.Tensor]:
        """Every fp32 state buffer in a fixed order: dense w, m, v, then per table w, m, v."""
        st = self.state
        out = [st.w, st.m, st.v]
        for t in self.tables.values():
            out += [t.w.view(-1), t.m.view(-1), t.v.view(-1)]
        return out

    def load(self, bufs, version, step, table_steps=None):
        for dst, src in zip(self.state_buffers(), bufs):
            dst.copy_(src.reshape(dst.shape))
        for t, k in zip(self.tables.values(), table_steps or []):
            t.step = int(k)
        self.version, self.step = int(version), int(step)

    def start(self) -> "ParameterServer":
        def accept():
            self._srv.settimeout(0.2)
            while not self._stop.is_set():
                try:
                    c, _ = self._srv.accept()
                except socket.timeout:
                    continue
                except OSError:
                    return
                c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                th = threading.Thread(target=self._serve, args=(c,), daemon=True)
                th.start()
                self._threads.append(th)

        t = threading.Thread(target=accept, name=f"edl-ps{self.index}", daemon=True)
        t.start()
        self._threads.append(t)
        return self

    def wait(self):
        while not self._stop.wait(0.2):
            pass

    def stop(self):
        self._stop.set()
        try:
            self._srv.close()
        except OSError:
            pass


# ---------------------------------------------------------------------------- snapshots
class PSSnapshotter:
    """Snapshot a PS shard into /dev/shm (A/B slots) and restore it in a replacement PS."""

    def __init__(self, job: str, index: int):
        self.name = f"/edl-{job}-ps{index}"
        self.seg = None
        self.engine = None
        self.ticket = None
        self._keep = None
        self._prep = None

    def prepare(self, ps: ParameterServer) -> None:
        """Create, pin and pre-fault the snapshot segment (and the copy engine) of an HBM shard
        on a background thread, so that the first snapshot does not stall the updates: mapping
        and pinning 2 x 4 GB (BERT-large) took seconds inside the first snapshot, while every
        worker's push waited (profiles/r05_ps_per_gpu.md)."""
        bufs = ps.state_buffers()
        if not bufs or not bufs[0].is_cuda or self.seg is not None:
            return
        nbytes = sum(b.numel() * 4 for b in bufs) + 8
        dev = bufs[0].device

        def run():
            from easydl_amd.ckpt.manager import CheckpointManager, ShmSegment
            try:
                torch.cuda.set_device(dev)
                seg = ShmSegment(self.name, nbytes, create=True, pin=True)
                seg.populate_async(8)
                self.engine = self.engine or CheckpointManager._make_engine(dev.index or 0)
                self.seg = seg
            except Exception as e:  # noqa: BLE001 - the first snapshot creates it then
                log.warning("PS snapshot segment preparation failed: %s", e)

        self._prep = threading.Thread(target=run, name="ps-snap-prep", daemon=True)
        self._prep.start()

    def __call__(self, ps: ParameterServer) -> None:
        from easydl_amd.ckpt.manager import ShmSegment, checksum_np
        if self._prep is not None:
            self._prep.join()
            self._prep = None
        bufs = ps.state_buffers()
        sizes = [b.numel() * 4 for b in bufs]
        total_bytes = sum(sizes)
        meta = {"sizes": sizes, "step": ps.step, "table_steps": [t.step for t in ps.tables.values()]}
        if bufs[0].is_cuda:
            self._snapshot_async(ps, bufs, sizes, meta)
            return
        if self.seg is None:
            self.seg = ShmSegment(self.name, total_bytes, create=True, pin=False)
        slot = self.seg.begin()
        total, off = 0, 0
        for buf, nb in zip(bufs, sizes):
            arr = buf.detach().cpu().contiguous().view(torch.uint8).numpy()
            self.seg.view(slot, off, nb)[:] = arr
            total += checksum_np(arr, off // 4)
            off += nb
        self.seg.commit(slot, ps.version, ps.step, off, total, meta)

    def _snapshot_async(self, ps: ParameterServer, bufs, sizes, meta) -> None:
        """HBM-resident shard: checksum on the GPU, D2H through the snapshot engine
        (CU-masked side stream, pinned segment, commit thread) — the PS keeps
        serving while the copy runs; the next update waits for it (fence)."""
        import ctypes
        import json

        from easydl_amd import _native
        from easydl_amd.ckpt.manager import CheckpointManager, ShmSegment, checksum_tensor
        rt = _native.runtime()
        dev = bufs[0].device
        cs_off = sum(sizes)
        if self.seg is None:
            self.seg = ShmSegment(self.name, cs_off + 8, create=True, pin=True)
        if self.engine is None:
            self.engine = CheckpointManager._make_engine(dev.index or 0)
        if self.ticket is not None:
            rt("edl_ckpt_wait", self.engine, self.ticket, 600000)  # at most one snapshot in flight
        csum = torch.zeros(1, dtype=torch.int64, device=dev)
        ptrs, offs, off = [], [], 0
        for b, nb in zip(bufs, sizes):
            checksum_tensor(b.view(-1), csum, base_index=off // 4)
            ptrs.append(b.data_ptr())
            offs.append(off)
            off += nb
        ptrs.append(csum.data_ptr())
        offs.append(cs_off)
        szs = list(sizes) + [8]
        n = len(ptrs)
        arr = lambda v: (ctypes.c_uint64 * n)(*v)  # noqa: E731
        t = rt("edl_ckpt_snapshot", self.engine, self.seg.h, n, arr(ptrs), arr(szs), arr(offs),
               ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream), ps.version, ps.step, cs_off,
               json.dumps(meta, separators=(",", ":")).encode())
        if t < 0:
            raise RuntimeError(f"PS snapshot enqueue failed: hipError {-t}")
        self.ticket, self._keep = t, csum

    def wait(self) -> None:
        """Block until the in-flight snapshot (GPU engine) is committed."""
        if self.ticket is not None and self.engine is not None:
            from easydl_amd import _native
            _native.runtime()("edl_ckpt_wait", self.engine, self.ticket, 600000)

    def fence(self, device) -> None:
        """The next update of the shard waits (on the GPU) for the in-flight copy."""
        if self.ticket is not None and self.engine is not None:
            import ctypes

            from easydl_amd import _native
            _native.runtime()("edl_ckpt_fence", self.engine, self.ticket,
                              ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream))

    def restore(self, ps: ParameterServer) -> bool:
        from easydl_amd.ckpt.manager import ShmSegment, checksum_np
        try:
            seg = ShmSegment(self.name, create=False)
        except OSError:
            return False
        try:
            infos = seg.committed()
            if not infos:
                return False
            info = max(infos, key=lambda i: i["step"])
            sizes = info["meta"].get("sizes")
            if sizes != [b.numel() * 4 for b in ps.state_buffers()]:
                return False
            bufs, total, off = [], 0, 0
            for nb in sizes:
                raw = seg.view(info["slot"], off, nb)
                total += checksum_np(raw, off // 4)
                bufs.append(torch.from_numpy(raw.copy()).view(torch.float32))
                off += nb
            if (total & ((1 << 64) - 1)) != info["checksum"]:
                log.error("PS snapshot checksum mismatch: ignoring")
                return False
            ps.load(bufs, info["step"], info["meta"]["step"], info["meta"].get("table_steps"))
            ps.stats["restored_version"] = ps.version
            return True
        finally:
            seg.close()

    def unlink(self):
        from easydl_amd.ckpt.manager import ShmSegment
        if self.seg is not None:
            self.seg.close(unlink=True)
            self.seg = None
