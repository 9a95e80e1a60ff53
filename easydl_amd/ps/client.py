"""Worker-side PS client + parameter partitioner.

Partitioning balances parameter bytes over the PS shards (largest tensors
first onto the least-loaded shard); it is a pure function of the model's
parameter names and sizes, so every role computes the same assignment without
coordination.  PS addresses are discovered through the job master's store
(``ps/addr/<i>``), and a client transparently reconnects when a PS is replaced
(new incarnation, new port).  A replaced GPU PS (reference "recover failed parameter
servers", /root/reference/README.md:27; replace-by-name, docs/design/elastic-training-operator.md:97-101)
is re-mapped over IPC: pushes in flight to the dead one are counted lost, never resent.
"""
from __future__ import annotations

import json
import os
import socket
import threading
import time
from concurrent.futures import ThreadPoolExecutor

import torch

from easydl_amd.ps.wire import connect, recv_msg, send_msg


def partition(named_sizes: list[tuple[str, int]], num_ps: int) -> dict[str, int]:
    load = [0] * num_ps
    out = {}
    for name, n in sorted(named_sizes, key=lambda x: (-x[1], x[0])):
        i = min(range(num_ps), key=lambda j: (load[j], j))
        out[name] = i
        load[i] += n
    return out


def dense_params(model: torch.nn.Module) -> dict[str, torch.Tensor]:
    """Named parameters that the PS serves densely (row-sparse PSEmbedding tables excluded)."""
    from easydl_amd.ps.embedding import tables_of
    skip = {f"{n}.weight" for n in tables_of(model)}
    return {n: p for n, p in model.named_parameters() if n not in skip}


def shard_of(model: torch.nn.Module, num_ps: int, index: int) -> dict[str, torch.Tensor]:
    params = dense_params(model)
    assign = partition([(n, p.numel()) for n, p in params.items()], num_ps)
    return {n: p.detach() for n, p in params.items() if assign[n] == index}


class PSReconnected(ConnectionError):
    """An IPC-bound request (``push_ipc``: its gradients sit in the OLD PS's mapped inbox) could
    not be delivered: the PS died and a replacement took its place.  Not re-sent -- the push is
    lost (async PS: counted in ``lost_pushes``); the client maps the replacement's buffers."""


class PSClient:
    def __init__(self, num_ps: int, resolve, worker_id: str, retry_s: float = 120.0, transport: str = "tcp"):
        """``resolve(i) -> (host, port)`` returns the current address of PS i.

        ``transport``: ``tcp`` (tensors over the socket) or ``ipc`` (GPU shards:
        parameters / gradients move through IPC-mapped HBM, easydl_amd/ps/ipc.py;
        TCP carries only control messages and sparse rows)."""
        self.num_ps = num_ps
        self.resolve = resolve
        self.worker_id = worker_id
        self.retry_s = retry_s
        self._socks: dict[int, socket.socket] = {}
        self._locks = [threading.Lock() for _ in range(num_ps)]
        self._pool = ThreadPoolExecutor(max_workers=max(1, num_ps))
        self.versions = [0] * num_ps
        self.assign: dict[str, int] = {}
        self.tables: dict = {}
        self.rows_bf16 = False  # pull embedding rows as bf16 (halves the wire bytes)
        self.transport = transport
        self._ipc: dict[int, dict] = {}   # PS index -> {"w", "inbox", "layout", "sock"}
        # GPU transport, row-sparse tables: rows per push a sparse inbox holds (a larger push
        # falls back to the TCP path for that step), per-table device pointer tables
        self.sparse_cap = int(os.environ.get("EDL_PS_SPARSE_CAP", 65536))
        self._sp_plan: dict = {}
        self.sparse_path = {"ipc_pulls": 0, "ipc_pushes": 0, "tcp_pulls": 0, "tcp_pushes": 0}
        self._inflight = None    # futures of the pipelined push in flight (push_async)
        # maps of a PS that died: kept until the device has drained every kernel that may still
        # read or write them (closing an IPC mapping under an in-flight kernel would fault)
        self._retired: list[dict] = []
        self.lost_pushes = [0] * num_ps
        self.reconnects: list[dict] = []  # {"ps", "lost", "version_before", "version_after", "s"}

    def bind(self, model: torch.nn.Module) -> None:
        from easydl_amd.ps.embedding import tables_of
        self.assign = partition([(n, p.numel()) for n, p in dense_params(model).items()], self.num_ps)
        self.tables = tables_of(model)
        for n, m in self.tables.items():
            m.attach(self, n)

    # -- row-sparse tables ---------------------------------------------------------
    def _split_rows(self, ids: torch.Tensor):
        ids = ids.reshape(-1).to(torch.int64)
        owner = ids % self.num_ps
        return [(i, (owner == i).nonzero().view(-1)) for i in range(self.num_ps)], ids

    def _sparse_ipc(self, device) -> bool:
        """Row-sparse traffic goes through the mapped tables / inboxes (no host copies)."""
        if self.transport != "ipc" or not self.tables or torch.device(device).type != "cuda":
            return False
        return all("tables" in self._ipc_map(i, device) for i in range(self.num_ps))

    def _table_ptrs(self, table: str, device):
        maps = [self._ipc_map(i, device) for i in range(self.num_ps)]
        key = ("tab", table, tuple(m["tables"][table][0].data_ptr() for m in maps))
        got = self._sp_plan.get(key[:2])
        if got is None or got[0] != key:
            from easydl_amd.ops.sparse import ptr_array
            tabs = ptr_array([m["tables"][table][0] for m in maps], device)
            nrows = torch.tensor([m["tables"][table][1] for m in maps], dtype=torch.int64).to(device)
            got = self._sp_plan[key[:2]] = (key, tabs, nrows)
        return got[1], got[2]

    def _inbox_ptrs(self, table: str, slots, device):
        maps = [self._ipc_map(i, device) for i in range(self.num_ps)]
        bufs = [m["sp_inbox"][table][s] for m, s in zip(maps, slots)]
        key = ("inbox", table, tuple(b[0].data_ptr() for b in bufs))
        got = self._sp_plan.get(key)
        if got is None:
            from easydl_amd.ops.sparse import ptr_array
            got = self._sp_plan[key] = tuple(ptr_array([b[k] for b in bufs], device) for k in range(3)) + (
                torch.zeros(max(4, self.num_ps), dtype=torch.int32, device=device),)
        return got

    def pull_rows(self, table: str, ids: torch.Tensor) -> torch.Tensor:
        """Rows ``ids`` (global) of ``table`` from their owning shards, fp32 [n, dim] on ids' device."""
        m = self.tables[table]
        if ids.is_cuda and self._sparse_ipc(ids.device):
            # one gather kernel reads every owner's mapped stripe (device-side owner split)
            from easydl_amd.ops.sparse import embed_gather_striped
            tabs, nrows = self._table_ptrs(table, ids.device)
            self.sparse_path["ipc_pulls"] += 1
            return embed_gather_striped(tabs, nrows, ids, m.dim)
        self.sparse_path["tcp_pulls"] += 1
        parts, flat = self._split_rows(ids.cpu())
        out = torch.empty(flat.numel(), m.dim, dtype=torch.float32)

        def one(arg):
            i, pos = arg
            if pos.numel() == 0:
                return
            h, ts = self._call(i, {"op": "pull_rows", "table": table, "bf16": self.rows_bf16},
                               {"ids": flat[pos] // self.num_ps})
            out[pos] = ts["rows"].float()

        list(self._pool.map(one, parts))
        return out.to(ids.device)

    def _sparse_grads(self, i: int, grads_by_table: dict) -> dict[str, torch.Tensor]:
        out = {}
        for n, (parts, flat, g) in grads_by_table.items():
            pos = parts[i][1]
            if pos.numel():
                out[f"sparse/{n}/ids"] = flat[pos] // self.num_ps
                out[f"sparse/{n}/grad"] = g[pos]
        return out

    def _call(self, i: int, header: dict, tensors=None, ipc_bound: bool = False):
        """One request to PS i; a broken connection is re-resolved and the request re-sent to
        the replacement PS -- unless it is ``ipc_bound`` (it refers to the dead PS's mapped
        buffers), which raises :class:`PSReconnected` instead."""
        t_end = time.monotonic() + self.retry_s
        while True:
            with self._locks[i]:
                try:
                    if i not in self._socks:
                        if ipc_bound and i not in self._ipc:
                            raise PSReconnected(f"PS {i}: mapping gone before {header.get('op')}")
                        self._socks[i] = connect(*self.resolve(i))
                    send_msg(self._socks[i], header, tensors)
                    h = recv_msg(self._socks[i])
                    if ipc_bound and isinstance(h[0], dict) and h[0].get("error") == "remap":
                        raise PSReconnected(f"PS {i} does not know this worker's mapping")
                    return h
                except PSReconnected:
                    self._retire_map(i)
                    raise
                except (ConnectionError, OSError, TimeoutError):
                    self._retire_map(i)     # a replacement PS exports new handles
                    s = self._socks.pop(i, None)
                    if s is not None:
                        try:
                            s.close()
                        except OSError:
                            pass
                    if ipc_bound:
                        raise PSReconnected(f"PS {i} connection lost during {header.get('op')}")
                    if time.monotonic() > t_end:
                        raise
            time.sleep(0.2)  # PS being replaced: re-resolve and retry

    def _retire_map(self, i: int) -> None:
        m = self._ipc.pop(i, None)
        if m is not None:
            self._retired.append(m)

    def _release_retired(self, device) -> None:
        """Drop dead PSs' mappings once no kernel of this process can still touch them.  Called
        only at the entry of pull / push (the thread that launches the copy kernels): the pool
        threads that notice a dead PS only move its map here, so a kernel the launching thread
        enqueued from that map keeps it referenced until this device-wide drain."""
        if self._retired and device is not None and torch.device(device).type == "cuda":
            torch.cuda.synchronize(device)
            self._retired.clear()

    def _remap_after_loss(self, i: int, device, t0: float) -> int:
        """The push to PS i was lost with its PS: map the replacement (which restored its newest
        snapshot and continues the version count from the highest version any worker saw) and
        go on from its current version."""
        before = self.versions[i]
        self.lost_pushes[i] += 1
        m = self._ipc_map(i, device)
        after = int(m.get("version", before))
        self.versions[i] = max(before, after)
        self.reconnects.append({"ps": i, "lost": 1, "version_before": before, "version_after": after,
                                "s": round(time.monotonic() - t0, 3)})
        return self.versions[i]

    # -- GPU transport ---------------------------------------------------------------
    # Bulk bytes never cross TCP: per PS, ONE kernel launch moves every parameter
    # (pull: fp32 shard -> this worker's bf16/fp32 params) or every gradient (push:
    # -> fp32, written into this worker's inbox in the PS's HBM).  Inboxes are double
    # buffered: push k writes inbox k % 2, and the PS answers push k only once the
    # update that read inbox (k - 1) % 2 has finished, so the next push may overwrite
    # it — the PS never blocks on the update it has just launched.
    def _ipc_map(self, i: int, device=None) -> dict:
        m = self._ipc.get(i)
        if m is None or m["sock"] is not self._socks.get(i):
            from easydl_amd.ps.ipc import import_tensor
            if m is not None:
                self._retire_map(i)
            # seen_version: a replacement PS continues the version count from the highest one
            # its workers saw, so no worker ever observes a version going back
            hdr = {"op": "ipc_open", "worker": self.worker_id, "sparse_cap": self.sparse_cap if self.tables else 0,
                   "seen_version": int(self.versions[i])}
            h, _ = self._call(i, hdr)
            if not h.get("ok"):
                raise RuntimeError(f"PS {i}: {h.get('error')}")
            d = h["ipc"]
            m = {"w": import_tensor(d["w"]), "inbox": [import_tensor(x) for x in d["inbox"]], "layout": d["layout"],
                 "sock": self._socks.get(i), "slot": 0, "pull_plan": None, "push_plan": None,
                 "flag": import_tensor(d["flag"]) if "flag" in d else None, "seq": 0,
                 "version": int(h.get("version", 0))}
            if "tables" in d:
                m["tables"] = {n: (import_tensor(x["w"]), int(x["rows"])) for n, x in d["tables"].items()}
                m["sp_inbox"] = {n: [[import_tensor(x) for x in b] for b in bufs]
                                 for n, bufs in d["sparse_inbox"].items()}
            self._ipc[i] = m
            self._sp_plan = {}
        return m

    @staticmethod
    def _plan(m: dict, which: str, tensors: list, device):
        """Cached MultiCopyPlan for this PS's layout (rebuilt if a tensor moved)."""
        from easydl_amd.ops.sparse import MultiCopyPlan
        key = tuple(0 if t is None else t.data_ptr() for t in tensors)
        plan = m[which]
        if plan is None or plan.key != key:
            items = [(t, off, int(torch.Size(shape).numel())) for t, (off, shape) in zip(tensors, m["layout"].values())]
            try:
                plan = MultiCopyPlan(items, device)
            except ValueError:
                plan = False      # odd layout / dtype: per-tensor copies
            m[which] = plan
        return plan or None

    def _pull_launch(self, i: int, params: dict) -> None:
        """Copy PS i's shard into the parameters on the current stream (one launch)."""
        m = self._ipc_map(i, next(iter(params.values())).device)
        ts = [params[n].data for n in m["layout"]]
        dev = ts[0].device
        plan = self._plan(m, "pull_plan", ts, dev)
        if plan is not None:
            plan.run(m["w"].data_ptr(), push=False)
            return
        from easydl_amd.ops.sparse import pull_cast
        w = m["w"]
        with torch.no_grad():
            for n, (off, shape) in m["layout"].items():
                p = params[n]
                k = p.numel()
                src = w[off:off + k]
                if p.dtype == torch.bfloat16 and k % 8 == 0 and p.is_contiguous():
                    pull_cast(src, p.view(-1))
                else:
                    p.copy_(src.view(p.shape))

    def _push_launch(self, i: int, params: dict) -> int:
        """Write this worker's gradients of PS i's shard into inbox ``slot``; returns the slot."""
        dev = next(iter(params.values())).device
        m = self._ipc_map(i, dev)
        slot = m["slot"]
        m["slot"] ^= 1
        inbox = m["inbox"][slot]
        gs = [params[n].grad for n in m["layout"]]
        plan = self._plan(m, "push_plan", gs, inbox.device if not gs or gs[0] is None else gs[0].device)
        if plan is not None:
            plan.run(inbox.data_ptr(), push=True)
            return slot
        with torch.no_grad():
            for (n, (off, shape)), g in zip(m["layout"].items(), gs):
                dst = inbox[off:off + params[n].numel()]
                if g is None:
                    dst.zero_()
                else:
                    dst.copy_(g.reshape(-1))
        return slot

    def _pull_ipc(self, i: int, params: dict, min_version=None) -> int:
        hdr = {"op": "pull_ipc"}
        if min_version is not None:
            hdr["min_version"] = min_version
        self._ipc_map(i, next(iter(params.values())).device)
        h, _ = self._call(i, hdr)
        return h["version"]

    def pull(self, model: torch.nn.Module, min_versions=None) -> list[int]:
        params = dict(model.named_parameters())
        self._release_retired(next(iter(params.values())).device)
        if self.transport == "ipc":
            # control round trips in parallel (version / bounded-staleness wait; the PS
            # answers once the update of that version has finished writing), then one
            # copy kernel per shard on this thread's stream (ordered before forward)
            self.versions = list(self._pool.map(
                lambda i: self._pull_ipc(i, params, None if min_versions is None else min_versions[i]),
                range(self.num_ps)))
            for i in range(self.num_ps):
                self._pull_launch(i, params)
            return self.versions

        def one(i):
            names = [n for n, j in self.assign.items() if j == i]
            hdr = {"op": "pull", "names": names}
            if min_versions is not None:
                hdr["min_version"] = min_versions[i]
            h, ts = self._call(i, hdr)
            with torch.no_grad():
                for n, t in ts.items():
                    params[n].copy_(t.to(params[n].device, params[n].dtype), non_blocking=True)
            return h["version"]

        self.versions = list(self._pool.map(one, range(self.num_ps)))
        return self.versions

    def _take_sparse(self) -> dict:
        sparse_grads = {}
        for n, m in self.tables.items():
            got = m.take_grads()
            if got is not None:
                parts, flat = self._split_rows(got[0].cpu())
                sparse_grads[n] = (parts, flat, got[1].detach().cpu())
        return sparse_grads

    def push(self, model: torch.nn.Module, step: int = 0, then_pull: bool = False) -> list[int]:
        """Push this step's gradients to every shard.  ``then_pull`` (GPU transport): the
        same round trip returns once the shard has applied them, and the fresh
        parameters are copied right away — push + pull in ONE control message per PS."""
        params = dict(model.named_parameters())
        self._release_retired(next(iter(params.values())).device)
        sparse_dev = {}
        if self.transport == "ipc" and self.tables:
            dev = next(iter(params.values())).device
            if self._sparse_ipc(dev):
                for n, mod in self.tables.items():
                    got = mod.take_grads()
                    if got is not None:
                        sparse_dev[n] = (got[0], got[1].detach())
                if any(ids.numel() > self.sparse_cap for ids, _ in sparse_dev.values()):
                    # larger than an inbox: this step's rows go over TCP
                    for n, (ids, g) in sparse_dev.items():
                        self.tables[n]._pending.append((ids, _Grad(g)))
                    sparse_dev = {}
        sparse_grads = {} if sparse_dev else self._take_sparse()
        if sparse_grads:
            self.sparse_path["tcp_pushes"] += 1

        if self.transport == "ipc":
            dev = next(iter(params.values())).device
            slots = [self._push_launch(i, params) for i in range(self.num_ps)]
            sp_ipc = bool(sparse_dev) or (bool(self.tables) and self._sparse_ipc(dev))
            if sp_ipc:
                # row-sparse gradients: split by owner on the device, written into each PS's
                # sparse inbox of this slot (every table, 0 rows included: the PS reads counts)
                from easydl_amd.ops.sparse import sparse_split_push
                for n, mod in self.tables.items():
                    ids, g = sparse_dev.get(n, (None, None))
                    iids, igrad, icnt, scratch = self._inbox_ptrs(n, slots, dev)
                    if ids is None:
                        ids = torch.empty(0, dtype=torch.int64, device=dev)
                        g = torch.empty(0, mod.dim, dtype=torch.float32, device=dev)
                    sparse_split_push(ids, g, iids, igrad, icnt, self.sparse_cap, scratch)
                self.sparse_path["ipc_pushes"] += 1
            seqs = [None] * self.num_ps
            stream = torch.cuda.current_stream(dev)
            if all(self._ipc[i].get("flag") is not None for i in range(self.num_ps)):
                # stream-ordered flag stores into each PS's HBM; the PS's stream waits for them
                # (bounded) before reading any inbox
                from easydl_amd.ops.sparse import ps_signal
                for i in range(self.num_ps):
                    m = self._ipc[i]
                    m["seq"] += 1
                    seqs[i] = m["seq"]
                    ps_signal(m["flag"], m["seq"], stream)
            # The control message leaves once this worker's stream has reached the flag stores
            # (each sender thread waits on the event; the main thread waits for the replies
            # anyway).  Sent earlier, it parks the PS's stream in its flag wait behind this
            # worker's backward, and every other worker's update queues behind that wait: in
            # config 4 ps_wait_kernel took 7.9 of a PS's 10.2 s of kernel time and the workers'
            # steady rate fell ~9 % (profiles/r04_bert_ps_flag_wait.md).  The device wait stays
            # as the ordering guard.
            ready = torch.cuda.Event()
            ready.record(stream)

            def one(i):
                ready.synchronize()
                hdr = {"op": "push_ipc", "worker": self.worker_id, "step": step, "slot": slots[i],
                       "pull": bool(then_pull), "sparse_ipc": sp_ipc, "seq": seqs[i]}
                t0 = time.monotonic()
                try:
                    h, _ = self._call(i, hdr, self._sparse_grads(i, sparse_grads), ipc_bound=True)
                except PSReconnected:
                    return self._remap_after_loss(i, dev, t0)
                return h["version"]

            self.versions = list(self._pool.map(one, range(self.num_ps)))
            if then_pull:
                for i in range(self.num_ps):
                    self._pull_launch(i, params)
            return self.versions

        def one(i):
            grads = self._sparse_grads(i, sparse_grads)
            for n, j in self.assign.items():
                if j == i:
                    g = params[n].grad
                    grads[n] = (g if g is not None else torch.zeros_like(params[n])).detach().float()
            h, _ = self._call(i, {"op": "push", "worker": self.worker_id, "step": step}, grads)
            return h["version"]

        self.versions = list(self._pool.map(one, range(self.num_ps)))
        if then_pull:
            self.pull(model)
        return self.versions

    # -- pipelined async pushes (bounded staleness) -------------------------------------
    # An async PS answers push k as soon as the update that read inbox (k - 1) % 2 has
    # finished and update k is launched.  So the worker need not wait for the answer before
    # its next step: it copies whatever the shard holds now (pull_local: at least the version
    # of push k - 2, usually k - 1) and sends push k + 1 once the answer to push k is in --
    # which is also what frees the inbox push k + 1 overwrites.  The PS's update of step k
    # then runs under the worker's step k + 1 instead of between the two.
    def pipelined(self) -> bool:
        return self.transport == "ipc" and not self.tables

    def push_async(self, model: torch.nn.Module, step: int = 0) -> None:
        """Enqueue this step's push (inbox copies and flag stores on the current stream) and
        send its control messages from the pool; returns at once.  Waits first for the
        previous push's answers (their inbox slot is the one this push writes)."""
        if not self.pipelined():
            raise RuntimeError("push_async needs the GPU transport and a dense model")
        self.drain()
        params = dict(model.named_parameters())
        self._release_retired(next(iter(params.values())).device)
        slots = [self._push_launch(i, params) for i in range(self.num_ps)]
        dev = next(iter(params.values())).device
        stream = torch.cuda.current_stream(dev)
        seqs = [None] * self.num_ps
        if all(self._ipc[i].get("flag") is not None for i in range(self.num_ps)):
            from easydl_amd.ops.sparse import ps_signal
            for i in range(self.num_ps):
                m = self._ipc[i]
                m["seq"] += 1
                seqs[i] = m["seq"]
                ps_signal(m["flag"], m["seq"], stream)
        ready = torch.cuda.Event()
        ready.record(stream)

        def one(i):
            ready.synchronize()     # the message leaves once the stream passed the flag stores
            hdr = {"op": "push_ipc", "worker": self.worker_id, "step": step, "slot": slots[i], "pull": False,
                   "sparse_ipc": False, "seq": seqs[i]}
            t0 = time.monotonic()
            try:
                h, _ = self._call(i, hdr, {}, ipc_bound=True)
            except PSReconnected:
                return self._remap_after_loss(i, dev, t0)
            return h["version"]

        self._inflight = [self._pool.submit(one, i) for i in range(self.num_ps)]

    def drain(self) -> list[int]:
        """Wait for the answers to the push in flight (if any); returns the shard versions."""
        fl, self._inflight = getattr(self, "_inflight", None), None
        if fl:
            self.versions = [f.result() for f in fl]
        return self.versions

    def pull_local(self, model: torch.nn.Module) -> None:
        """Copy every shard's current parameters into ``model`` (one kernel per shard on the
        current stream, no control message).  Async semantics: an update of the shard may be
        running meanwhile, so the copy holds each parameter word of version >= the last
        answered push - 1."""
        params = dict(model.named_parameters())
        self._release_retired(next(iter(params.values())).device)
        for i in range(self.num_ps):
            self._pull_launch(i, params)

    def stats(self) -> list[dict]:
        return [self._call(i, {"op": "stats"})[0] for i in range(self.num_ps)]

    def close(self):
        try:
            self.drain()
        except Exception:  # noqa: BLE001 - closing: the PS may be gone
            pass
        for s in self._socks.values():
            try:
                s.close()
            except OSError:
                pass
        self._socks.clear()
        self._pool.shutdown(wait=False)


def store_resolver(kv, timeout_s: float = 300.0):
    def resolve(i: int):
        t_end = time.monotonic() + timeout_s
        while time.monotonic() < t_end:
            a = kv.get(f"ps/addr/{i}")
            if a:
                a = a if isinstance(a, dict) else json.loads(a)
                return a["host"], int(a["port"])
            time.sleep(0.1)
        raise TimeoutError(f"PS {i} address not published")

    return resolve


class _Grad:
    """Stands in for a leaf whose ``.grad`` holds already de-duplicated row gradients."""

    def __init__(self, g):
        self.grad = g
