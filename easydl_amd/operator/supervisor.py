"""Python face of the native process supervisor (csrc/runtime/supervisor.cpp).

``spawn`` returns a pid; ``poll(timeout)`` returns exit events as soon as a
child dies (pidfd + epoll in C++: crash / OOM kill / ``kill -9`` are seen in
microseconds — the "detect" phase of time-to-recover).
"""
from __future__ import annotations

import ctypes
import os
import signal
import time
from dataclasses import dataclass

from easydl_amd import _native
from easydl_amd._runtime_sigs import ExitEvent


@dataclass
class Exit:
    pid: int
    name: str
    exit_code: int
    signal: int
    ts: float

    @property
    def ok(self) -> bool:
        return self.signal == 0 and self.exit_code == 0

    def describe(self) -> str:
        return f"signal {self.signal}" if self.signal else f"exit {self.exit_code}"


class Supervisor:
    def __init__(self):
        self.rt = _native.runtime()
        self.h = self.rt("edl_sup_create")
        if not self.h:
            raise OSError("edl_sup_create failed")
        self.names: dict[int, str] = {}

    def spawn(self, name: str, argv: list[str], env: dict | None = None, cwd: str | None = None,
              log_path: str | None = None, cpus: list[int] | None = None, new_pgrp: bool = True) -> int:
        exe = argv[0]
        if os.sep not in exe:
            import shutil
            found = shutil.which(exe)
            if found is None:
                raise FileNotFoundError(exe)
            exe = found
        args = [exe] + list(argv[1:])
        c_argv = (ctypes.c_char_p * (len(args) + 1))(*[a.encode() for a in args], None)
        envl = None
        if env is not None:
            items = [f"{k}={v}".encode() for k, v in env.items()]
            envl = (ctypes.c_char_p * (len(items) + 1))(*items, None)
        cpus = cpus or []
        c_cpus = (ctypes.c_int * max(1, len(cpus)))(*cpus) if cpus else (ctypes.c_int * 1)(0)
        pid = ctypes.c_int(0)
        if log_path:
            os.makedirs(os.path.dirname(os.path.abspath(log_path)), exist_ok=True)
        rc = self.rt("edl_sup_spawn", self.h, name.encode(), c_argv, envl, (cwd or "").encode(),
                     (log_path or "").encode(), c_cpus, len(cpus), 1 if new_pgrp else 0, ctypes.byref(pid))
        if rc != 0:
            raise OSError(-rc, f"spawn {name} failed: {os.strerror(-rc)}")
        self.names[pid.value] = name
        return pid.value

    def poll(self, timeout_s: float = 0.0, max_events: int = 64) -> list[Exit]:
        buf = (ExitEvent * max_events)()
        n = self.rt("edl_sup_wait", self.h, int(timeout_s * 1000), buf, max_events)
        if n < 0:
            raise OSError(-n, "edl_sup_wait failed")
        out = []
        for i in range(n):
            e = buf[i]
            out.append(Exit(e.pid, self.names.pop(e.pid, "?"), e.exit_code, e.signal, e.ts_ns / 1e9))
        return out

    def exiting(self, max_n: int = 64) -> list[int]:
        """Children already inside exit() (PF_EXITING) but not yet reaped."""
        buf = (ctypes.c_int * max_n)()
        n = self.rt("edl_sup_exiting", self.h, buf, max_n)
        return [buf[i] for i in range(max(0, n))]

    def kill(self, pid: int, sig: int = signal.SIGKILL, group: bool = True) -> None:
        rc = self.rt("edl_sup_kill", self.h, pid, int(sig), 1 if group else 0)
        if rc != 0 and -rc != 3:  # ESRCH: already gone
            raise OSError(-rc, f"kill {pid}")

    def terminate(self, pid: int, grace_s: float = 5.0) -> list[Exit]:
        """SIGTERM, then SIGKILL after ``grace_s``; returns exit events seen meanwhile."""
        self.kill(pid, signal.SIGTERM)
        seen = []
        t_end = time.monotonic() + grace_s
        while pid in self.names and time.monotonic() < t_end:
            seen += self.poll(0.05)
        if pid in self.names:
            self.kill(pid, signal.SIGKILL)
            t_end = time.monotonic() + 5
            while pid in self.names and time.monotonic() < t_end:
                seen += self.poll(0.05)
        return seen

    def alive(self) -> dict[int, str]:
        return dict(self.names)

    def close(self) -> None:
        if self.h:
            self.rt("edl_sup_destroy", self.h)
            self.h = None
            self.names.clear()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
