"""Tensor parallel Llama (TP=2 over gloo) == dense model: loss and every sharded grad."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("sp", ["0", "1"])
def test_tp2_matches_dense(tmp_path, sp):
    """sp=1: Megatron sequence parallelism (token-sharded residual stream and norms)."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "tests/helpers/tp_worker.py")],
                              env=dict(os.environ, RANK=str(r), WORLD_SIZE="2", PORT=str(port),
                                       OUT=str(tmp_path / "r"), PYTHONPATH=ROOT, SP=sp)) for r in range(2)]
    assert [p.wait(timeout=120) for p in procs] == [0, 0]
    for r in range(2):
        res = json.load(open(tmp_path / f"r.{r}"))
        assert abs(res["loss_d"] - res["loss_t"]) < 1e-5, res
        assert res["grad_rel_err"] < 1e-4, res
