"""bench.py contract (the driver's launch form) on CPU: N=2 ranks under
torch.distributed.run over gloo, a tiny Llama, one JSON line from rank 0 with
the fields the driver reads.  The GPU run of the same file is the round-end bench."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_two_ranks_prints_one_json_line(tmp_path):
    env = dict(os.environ, OMP_NUM_THREADS="2", EDL_RUN_DIR=str(tmp_path / "run"))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2", "--steps", "2",
           "--warmup", "1", "--model", "llama-tiny", "--seq", "64", "--mbs", "1", "--accum", "2"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in d, k
    assert d["n_gpus"] == 2 and d["steps"] == 2 and d["warmup"] == 1 and d["value"] > 0
    assert d["config"]["parallelism"] == "dp2" and d["config"]["global_batch"] == 4
    # value is the whole-job aggregate: 2 ranks x 1 seq x 64 tokens x 2 micro-batches per step
    assert abs(d["value"] - 2 * 64 * 2 * 2 / (d["ms_per_step"] * 2 / 1e3)) / d["value"] < 0.01
