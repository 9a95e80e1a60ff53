"""EDL_CHECK_COLLECTIVES=1: ranks that issue different collectives at the same
position fail fast with CollectiveMismatch instead of hanging or silently
reducing mismatched buffers (SURVEY.md §5.2 race/mismatch detection)."""
import datetime
import socket
import threading

import torch
import torch.distributed as dist

from easydl_amd.parallel.comm import CollectiveMismatch, Communicator


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(sizes_by_rank, monkeypatch):
    monkeypatch.setenv("EDL_CHECK_COLLECTIVES", "1")
    port = _port()
    out = {}

    def rank(r):
        st = dist.TCPStore("127.0.0.1", port, 2, r == 0, timeout=datetime.timedelta(seconds=30))
        c = Communicator(st, r, 2, 1, device=torch.device("cpu"), job="chk", timeout_s=20, control_timeout_s=20)
        try:
            for n in sizes_by_rank[r]:
                c.all_reduce(torch.ones(n))
            out[r] = "ok"
        except CollectiveMismatch as e:
            out[r] = f"mismatch: {e}"

    ts = [threading.Thread(target=rank, args=(r,)) for r in range(2)]
    [t.start() for t in ts]
    [t.join(60) for t in ts]
    return out


def test_matching_sequences_pass(monkeypatch):
    assert _run({0: [8, 16, 4], 1: [8, 16, 4]}, monkeypatch) == {0: "ok", 1: "ok"}


def test_mismatched_bucket_is_reported_on_every_rank(monkeypatch):
    out = _run({0: [8, 16, 4], 1: [8, 12, 4]}, monkeypatch)
    assert out[0].startswith("mismatch") and out[1].startswith("mismatch"), out
    assert "#2" in out[0]
