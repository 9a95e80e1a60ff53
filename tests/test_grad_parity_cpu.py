"""VERDICT r5 Weak #8: gradient precision at world > 1.  With bf16 gradient buffers the bucketed
all-reduce sums in bf16 (RCCL rounds at every hop; gloo here, the same arithmetic), while the xGMI
engine accumulates in fp32.  Eight gloo ranks train llama-tiny for 50 steps with bf16 and with fp32
gradient buffers; a single rank with bf16 buffers (the same 16 samples per step, accumulated over 16
micro-batches instead of 2 + an 8-rank sum) separates the all-reduce's share of the rounding.

Measured (printed): the drift of the bf16 runs from the fp32 run, relative to how far the weights
moved.  The test pins that the 8-rank bf16 all-reduce adds no material drift beyond bf16 gradient
accumulation itself -- the reason bf16 stays the default bucket dtype (half the xGMI bytes)."""
import os
import socket
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HELPER = os.path.join(ROOT, "tests", "helpers", "grad_parity_worker.py")


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(tmp, grad: str, n: int) -> dict:
    out = tmp / f"{grad}-{n}.pt"
    env = dict(os.environ, OMP_NUM_THREADS="1", EDL_RUN_DIR=str(tmp / f"run-{grad}-{n}"), PYTHONPATH=ROOT)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "EDL_MASTER_ADDR"):
        env.pop(k, None)
    if n == 1:
        cmd = [sys.executable, HELPER, grad, str(out)]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
               "--master-addr", "127.0.0.1", "--master-port", str(_port()), HELPER, grad, str(out)]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=420)
    assert r.returncode == 0, r.stderr[-3000:]
    return torch.load(out, weights_only=True)


@pytest.mark.slow
def test_bf16_allreduce_at_world8_adds_no_material_drift(tmp_path):
    ref = _run(tmp_path, "fp32", 8)
    bf8 = _run(tmp_path, "bf16", 8)
    bf1 = _run(tmp_path, "bf16", 1)
    assert ref["world"] == 8 and bf8["world"] == 8 and bf1["world"] == 1
    assert torch.equal(ref["init"], bf8["init"]) and torch.equal(ref["init"], bf1["init"])
    moved = (ref["final"] - ref["init"]).norm()
    d8 = float((bf8["final"] - ref["final"]).norm() / moved)
    d1 = float((bf1["final"] - ref["final"]).norm() / moved)
    dl8 = abs(bf8["losses"][-1] - ref["losses"][-1]) / ref["losses"][-1]
    print(f"\n[grad-parity] weights moved {float(moved):.4f}; drift from fp32 after 50 steps: "
          f"bf16 8 ranks {d8:.4%}, bf16 1 rank {d1:.4%}; final loss fp32 {ref['losses'][-1]:.4f} "
          f"bf16x8 {bf8['losses'][-1]:.4f} ({dl8:.3%})")
    assert d8 < 0.05, d8                    # < 5 % of the distance trained
    assert d8 < 2.0 * d1 + 0.005, (d8, d1)  # the 8-rank bf16 sum is not the material part
    assert dl8 < 0.01
