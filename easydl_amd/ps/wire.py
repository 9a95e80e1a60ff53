"""Length-prefixed tensor messages over TCP for the parameter-server plane.

Frame: ``u32 header_len | header JSON | payload`` where the header lists
``tensors: [{name, dtype, shape, nbytes}]`` and the payload is their raw bytes
back to back.  Tensors are sent straight from their (CPU) memory with
``sendall(memoryview)`` and received with ``recv_into`` a preallocated buffer
— no pickling anywhere (nothing executable crosses the wire).
"""
from __future__ import annotations

import json
import socket
import struct

import torch

_DT = {torch.float32: "f32", torch.bfloat16: "bf16", torch.float16: "f16", torch.int64: "i64", torch.int32: "i32",
       torch.uint8: "u8"}
_TD = {v: k for k, v in _DT.items()}


def _as_bytes(t: torch.Tensor) -> memoryview:
    t = t.detach()
    if t.is_cuda:
        t = t.cpu()
    t = t.contiguous()
    return memoryview(t.view(torch.uint8).numpy()).cast("B")


def send_msg(sock: socket.socket, header: dict, tensors: dict[str, torch.Tensor] | None = None) -> None:
    tensors = tensors or {}
    metas, views = [], []
    for name, t in tensors.items():
        mv = _as_bytes(t)
        metas.append({"name": name, "dtype": _DT[t.dtype], "shape": list(t.shape), "nbytes": mv.nbytes})
        views.append(mv)
    h = dict(header)
    h["tensors"] = metas
    hb = json.dumps(h, separators=(",", ":")).encode()
    sock.sendall(struct.pack("<I", len(hb)) + hb)
    for mv in views:
        if mv.nbytes:
            sock.sendall(mv)


def _recv_exact(sock: socket.socket, n: int) -> bytearray:
    buf = bytearray(n)
    view = memoryview(buf)
    got = 0
    while got < n:
        k = sock.recv_into(view[got:], n - got)
        if k == 0:
            raise ConnectionError("peer closed")
        got += k
    return buf


def recv_msg(sock: socket.socket) -> tuple[dict, dict[str, torch.Tensor]]:
    (hl,) = struct.unpack("<I", bytes(_recv_exact(sock, 4)))
    header = json.loads(bytes(_recv_exact(sock, hl)).decode())
    out = {}
    for m in header.get("tensors", []):
        raw = _recv_exact(sock, m["nbytes"]) if m["nbytes"] else bytearray()
        t = torch.frombuffer(raw, dtype=torch.uint8) if m["nbytes"] else torch.empty(0, dtype=torch.uint8)
        out[m["name"]] = t.view(_TD[m["dtype"]]).reshape(m["shape"])
    return header, out


def connect(host: str, port: int, timeout_s: float = 30.0) -> socket.socket:
    s = socket.create_connection((host, port), timeout=timeout_s)
    s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
    s.settimeout(None)
    return s
