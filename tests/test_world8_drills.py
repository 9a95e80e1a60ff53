"""World-8 paths on the CPU tier (VERDICT r4 "Next" #2): the exact launch forms the driver
and an 8-GPU node will use, rehearsed with 8 CPU processes over gloo.

* ``bench.py --fault-inject --gpus 8``: 8 workers + 1 hot standby under the local operator;
  one worker is SIGKILLed mid-step -> the 7 survivors shrink and go on -> the standby takes
  the dead worker's place and rejoins -> world 8 again.  No hang, <= 1 step lost, and every
  one of the 8 final ranks holds bit-identical parameters.
* ``torch.distributed.run --nproc-per-node 8 bench.py --gpus 8``: the driver's N=8 form.
"""
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


def _json_line(out: str) -> dict:
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out[-3000:]
    return json.loads(lines[0])


def test_fault_drill_world8_kill_shrink_rejoin(tmp_path):
    env = dict(os.environ, OMP_NUM_THREADS="1", EDL_TTR_DIR=str(tmp_path), EDL_BENCH_UNTIL_REGROWN="1",
               EDL_BENCH_CAP="3000", EDL_FAULT_STEP_MS="50")
    cmd = [sys.executable, "bench.py", "--fault-inject", "--gpus", "8", "--fault-mode", "midstep", "--standby", "1",
           "--fault-step", "3", "--steps", "0", "--warmup", "0"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=420)
    assert r.returncode == 0, r.stderr[-4000:]
    d = _json_line(r.stdout)
    assert d["operator_rc"] == 0 and d["workers"] == 8 and d["replacement_from_standby"]
    assert d["value"] is not None and d["value"] < 30, d["breakdown"]
    assert d["steps_lost"] is not None and d["steps_lost"] <= 1
    assert 7 in d["worlds_seen"] and 8 in d["worlds_seen"], d["worlds_seen"]
    finals = d["final_states"]
    assert len(finals) == 8, finals
    assert {f["world"] for f in finals} == {8} and sorted(f["rank"] for f in finals) == list(range(8))
    assert len({f["step"] for f in finals}) == 1
    assert len({json.dumps(f["crc"]) for f in finals}) == 1, finals     # identical parameters everywhere


def test_bench_eight_ranks_under_torchrun(tmp_path):
    env = dict(os.environ, OMP_NUM_THREADS="1", EDL_RUN_DIR=str(tmp_path / "run"))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "8", "--steps", "2",
           "--warmup", "1", "--model", "llama-tiny", "--seq", "64", "--mbs", "1", "--accum", "2"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=420)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 8 and d["steps"] == 2 and d["warmup"] == 1 and d["value"] > 0
    assert d["config"]["parallelism"] == "dp8" and d["config"]["global_batch"] == 16
    assert abs(d["value"] - 8 * 64 * 2 * 2 / (d["ms_per_step"] * 2 / 1e3)) / d["value"] < 0.01
