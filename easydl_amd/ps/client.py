"""Worker-side PS client + parameter partitioner.

Partitioning balances parameter bytes over the PS shards (largest tensors
first onto the least-loaded shard); it is a pure function of the model's
parameter names and sizes, so every role computes the same assignment without
coordination.  PS addresses are discovered through the job master's store
(``ps/addr/<i>``), and a client transparently reconnects when a PS is replaced
(new incarnation, new port).
"""
from __future__ import annotations

import json
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

    def pull_rows(self, table: str, ids: torch.Tensor) -> torch.Tensor:
        """Rows ``ids`` (global) of ``table`` from their owning shards, fp32 [n, dim] on ids' device."""
        m = self.tables[table]
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

    def _call(self, i: int, header: dict, tensors=None):
        t_end = time.monotonic() + self.retry_s
        while True:
            with self._locks[i]:
                try:
                    if i not in self._socks:
                        self._socks[i] = connect(*self.resolve(i))
                    send_msg(self._socks[i], header, tensors)
                    return recv_msg(self._socks[i])
                except (ConnectionError, OSError, TimeoutError):
                    self._ipc.pop(i, None)  # a replacement PS exports new handles
                    s = self._socks.pop(i, None)
                    if s is not None:
                        try:
                            s.close()
                        except OSError:
                            pass
                    if time.monotonic() > t_end:
                        raise
            time.sleep(0.2)  # PS being replaced: re-resolve and retry

    # -- GPU transport ---------------------------------------------------------------
    def _ipc_map(self, i: int) -> dict:
        m = self._ipc.get(i)
        if m is None or m["sock"] is not self._socks.get(i):
            from easydl_amd.ps.ipc import import_tensor
            h, _ = self._call(i, {"op": "ipc_open", "worker": self.worker_id})
            if not h.get("ok"):
                raise RuntimeError(f"PS {i}: {h.get('error')}")
            d = h["ipc"]
            m = {"w": import_tensor(d["w"]), "inbox": import_tensor(d["inbox"]), "layout": d["layout"],
                 "sock": self._socks.get(i)}
            self._ipc[i] = m
        return m

    def _pull_ipc(self, i: int, params: dict, min_version=None) -> int:
        from easydl_amd.ops.sparse import pull_cast
        hdr = {"op": "pull_ipc"}
        if min_version is not None:
            hdr["min_version"] = min_version
        m = self._ipc_map(i)
        h, _ = self._call(i, hdr)
        w = m["w"]
        with torch.no_grad():
            for n, (off, shape) in m["layout"].items():
                p = params[n]
                k = p.numel()
                src = w[off:off + k]
                if p.dtype == torch.bfloat16 and k % 8 == 0 and p.is_contiguous():
                    pull_cast(src, p.view(-1))   # HIP kernel on this GPU, fp32 read from the PS's HBM
                else:
                    p.copy_(src.view(p.shape))
        torch.cuda.current_stream(next(iter(params.values())).device).synchronize()
        return h["version"]

    def _push_ipc(self, i: int, params: dict, extra: dict, step: int) -> int:
        m = self._ipc_map(i)
        inbox = m["inbox"]
        with torch.no_grad():
            for n, (off, shape) in m["layout"].items():
                g = params[n].grad
                dst = inbox[off:off + params[n].numel()]
                if g is None:
                    dst.zero_()
                else:
                    dst.copy_(g.reshape(-1))  # peer writes into the PS's HBM
        torch.cuda.current_stream(next(iter(params.values())).device).synchronize()
        h, _ = self._call(i, {"op": "push_ipc", "worker": self.worker_id, "step": step}, extra)
        return h["version"]

    def pull(self, model: torch.nn.Module, min_versions=None) -> list[int]:
        params = dict(model.named_parameters())
        if self.transport == "ipc":
            self.versions = list(self._pool.map(
                lambda i: self._pull_ipc(i, params, None if min_versions is None else min_versions[i]),
                range(self.num_ps)))
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

    def push(self, model: torch.nn.Module, step: int = 0) -> list[int]:
        params = dict(model.named_parameters())
        sparse_grads = {}
        for n, m in self.tables.items():
            got = m.take_grads()
            if got is not None:
                parts, flat = self._split_rows(got[0].cpu())
                sparse_grads[n] = (parts, flat, got[1].detach().cpu())

        if self.transport == "ipc":
            self.versions = list(self._pool.map(
                lambda i: self._push_ipc(i, params, self._sparse_grads(i, sparse_grads), step), range(self.num_ps)))
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
        return self.versions

    def stats(self) -> list[dict]:
        return [self._call(i, {"op": "stats"})[0] for i in range(self.num_ps)]

    def close(self):
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
