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
import threading
import time

import torch

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


class ParameterServer:
    def __init__(self, index: int, tensors: dict[str, torch.Tensor], *, optimizer: str = "adam", lr: float = 1e-3,
                 betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0, momentum: float = 0.9,
                 mode: str = "async", expected_workers=None, host: str = "127.0.0.1", port: int = 0,
                 device="cpu", snapshot=None, snapshot_every: int = 50):
        self.index = index
        self.state = ShardState(tensors, device)
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
        self._srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self._srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self._srv.bind((host, port))
        self._srv.listen(128)
        self.host, self.port = self._srv.getsockname()
        self._stop = threading.Event()
        self._threads = []

    # -- optimizer -------------------------------------------------------------
    def _apply(self, scale: float) -> None:
        st = self.state
        self.step += 1
        if self.optimizer == "adam":
            adamw_flat_(None, st.w, st.m, st.v, st.g, lr=self.lr, beta1=self.betas[0], beta2=self.betas[1],
                        eps=self.eps, weight_decay=self.wd, step=self.step, scale=scale)
        else:
            sgd_flat_(None, st.w, st.m if self.momentum else None, st.g, lr=self.lr, momentum=self.momentum,
                      weight_decay=self.wd, scale=scale)
        st.g.zero_()
        self.version += 1
        self.stats["applied"] += 1
        if self.snapshot is not None and self.version % self.snapshot_every == 0:
            self.snapshot(self)
        self.lock.notify_all()

    def _push(self, worker: str, grads: dict[str, torch.Tensor]) -> int:
        with self.lock:
            st = self.state
            for n, g in grads.items():
                st.view(st.g, n).add_(g.to(st.device, torch.float32))
            self.stats["pushes"] += 1
            self.stats["workers"].add(worker)
            if self.mode == "async":
                self._apply(1.0)
                return self.version
            # sync: one contribution per worker per round
            self.round_pushers.add(worker)
            target = self.version + 1
            while self.version < target:
                if len(self.round_pushers) >= max(1, self.expected_workers()):
                    n = len(self.round_pushers)
                    self.round_pushers = set()
                    self._apply(1.0 / n)
                    break
                if not self.lock.wait(timeout=0.05):
                    continue
            return self.version

    # -- serving ---------------------------------------------------------------
    def _serve(self, conn: socket.socket):
        try:
            while not self._stop.is_set():
                try:
                    hdr, tensors = recv_msg(conn)
                except (ConnectionError, OSError):
                    return
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
                elif op == "push":
                    ver = self._push(hdr.get("worker", "?"), tensors)
                    send_msg(conn, {"ok": True, "version": ver})
                elif op == "state":
                    with self.lock:
                        st = self.state
                        out = {"w": st.w.clone(), "m": st.m.clone(), "v": st.v.clone()}
                        meta = {"version": self.version, "step": self.step}
                    send_msg(conn, {"ok": True, **meta}, out)
                elif op == "load":
                    with self.lock:
                        self.load(tensors["w"], tensors["m"], tensors["v"], hdr["version"], hdr["step"])
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
        finally:
            conn.close()

    def load(self, w, m, v, version, step):
        st = self.state
        st.w.copy_(w)
        st.m.copy_(m)
        st.v.copy_(v)
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

    def __call__(self, ps: ParameterServer) -> None:
        from easydl_amd.ckpt.manager import ShmSegment, checksum_np
        st = ps.state
        nbytes = st.w.numel() * 4
        if self.seg is None:
            self.seg = ShmSegment(self.name, 3 * nbytes, create=True, pin=False)
        slot = self.seg.begin()
        total = 0
        for i, buf in enumerate((st.w, st.m, st.v)):
            arr = buf.detach().cpu().contiguous().view(torch.uint8).numpy()
            self.seg.view(slot, i * nbytes, nbytes)[:] = arr
            total += checksum_np(arr, i * nbytes // 4)
        self.seg.commit(slot, ps.version, ps.step, 3 * nbytes, total, {"n": st.w.numel(), "step": ps.step})

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
            n = info["meta"]["n"]
            if n != ps.state.w.numel():
                return False
            nbytes = n * 4
            bufs, total = [], 0
            for i in range(3):
                raw = seg.view(info["slot"], i * nbytes, nbytes)
                total += checksum_np(raw, i * nbytes // 4)
                bufs.append(torch.from_numpy(raw.copy()).view(torch.float32))
            if (total & ((1 << 64) - 1)) != info["checksum"]:
                log.error("PS snapshot checksum mismatch: ignoring")
                return False
            ps.load(*bufs, info["step"], info["meta"]["step"])
            return True
        finally:
            seg.close()

    def unlink(self):
        from easydl_amd.ckpt.manager import ShmSegment
        if self.seg is not None:
            self.seg.close(unlink=True)
            self.seg = None
