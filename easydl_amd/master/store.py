"""Thin typed helpers over a c10d key-value store (TCPStore / HashStore).

The job master hosts a ``TCPStore`` server; every control-plane exchange
(rendezvous, heartbeats, commit votes, exit events, data-dispatch cursors,
metrics, plans) is a key under ``edl/<job>/``.  No protoc/gRPC exists in this
environment, so the store *is* the RPC substrate, which
also keeps the control plane free of extra daemons.
"""
from __future__ import annotations

import datetime
import json
import time

import torch.distributed as dist


class KV:
    def __init__(self, store: dist.Store, prefix: str = ""):
        self.raw = store
        self.prefix = prefix.rstrip("/")
        self.store = dist.PrefixStore(self.prefix, store) if self.prefix else store

    def sub(self, name: str) -> "KV":
        return KV(self.raw, f"{self.prefix}/{name}" if self.prefix else name)

    # -- scalars -----------------------------------------------------------------
    def set(self, key: str, value) -> None:
        if not isinstance(value, (bytes, str)):
            value = json.dumps(value)
        self.store.set(key, value)

    def get(self, key: str, default=None):
        if not self.exists(key):
            return default
        v = self.store.get(key)
        try:
            return json.loads(v)
        except (ValueError, UnicodeDecodeError):
            return v.decode() if isinstance(v, bytes) else v

    def get_str(self, key: str, default: str | None = None) -> str | None:
        if not self.exists(key):
            return default
        v = self.store.get(key)
        return v.decode() if isinstance(v, bytes) else v

    def exists(self, key: str) -> bool:
        return self.store.check([key])

    def delete(self, key: str) -> None:
        try:
            self.store.delete_key(key)
        except Exception:
            pass

    def add(self, key: str, n: int = 1) -> int:
        return int(self.store.add(key, n))

    def counter(self, key: str) -> int:
        """Read an integer counter without modifying it (0 if absent)."""
        return int(self.store.add(key, 0))

    def append(self, key: str, value: str) -> None:
        self.store.append(key, value)

    def compare_set(self, key: str, expected: str, desired: str) -> str:
        r = self.store.compare_set(key, expected, desired)
        return r.decode() if isinstance(r, bytes) else r

    def wait_for(self, key: str, timeout_s: float, poll_s: float = 0.002, abort=None) -> bool:
        """Poll until ``key`` exists; ``abort()`` returning True stops early."""
        t_end = time.monotonic() + timeout_s
        while time.monotonic() < t_end:
            if self.exists(key):
                return True
            if abort is not None and abort():
                return False
            time.sleep(poll_s)
        return False


def make_tcp_store(host: str, port: int, is_server: bool, world_size: int | None = None,
                   timeout_s: float = 300.0) -> dist.TCPStore:
    return dist.TCPStore(host, port, world_size, is_server, timeout=datetime.timedelta(seconds=timeout_s),
                         wait_for_workers=False, multi_tenant=False)
