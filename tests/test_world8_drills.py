"""World-8 paths on the CPU tier (VERDICT r4 "Next" #2): the exact launch forms the driver
and an 8-GPU node will use, rehearsed with 8 CPU processes over gloo.

* ``bench.py --gpus 8`` (plain): the parent launches 8 ranks for the throughput line, then
  8 workers + 1 hot standby under the local operator; one worker is SIGKILLed mid-step -> the
  7 survivors shrink and go on -> the standby takes the dead worker's place and rejoins ->
  world 8 again.  No hang, <= 1 step lost, and every one of the 8 final ranks holds
  bit-identical parameters; throughput and TTR in one JSON line.
* ``torch.distributed.run --nproc-per-node 8 bench.py --gpus 8``: the driver's N=8 form
  (throughput, with ``ttr.error`` naming the plain form).
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


def test_plain_bench_eight_ranks_reports_throughput_and_ttr(tmp_path):
    """The headline command at N = 8 without a launcher: bench.py's GPU-free parent starts the 8
    rank processes itself, then the 8-worker drill (SIGKILL of one worker mid-step -> 7 survivors
    shrink and go on -> the hot standby rejoins -> world 8), all in one JSON line."""
    env = dict(os.environ, OMP_NUM_THREADS="1", EDL_TTR_DIR=str(tmp_path), EDL_BENCH_CAP="3000",
               EDL_RUN_DIR=str(tmp_path / "run"))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, "bench.py", "--gpus", "8", "--model", "llama-tiny", "--seq", "64", "--mbs", "1",
           "--accum", "2", "--steps", "2", "--warmup", "1"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 8 and d["config"]["parallelism"] == "dp8" and d["steps"] == 2 and d["warmup"] == 1
    assert d["value"] > 0 and d["config"]["global_batch"] == 16
    t = d["ttr"]
    assert d["time_to_recover_s"] is not None and d["time_to_recover_s"] < 30, t
    assert t["operator_rc"] == 0 and t["workers"] == 8 and t["replacement_from_standby"], t
    assert 7 in t["worlds_seen"] and 8 in t["worlds_seen"], t["worlds_seen"]
    assert t["steps_lost"] is not None and t["steps_lost"] <= 1
    assert t["time_to_regrow_s"] is not None and t["time_to_regrow_s"] >= d["time_to_recover_s"]
    assert t["final_ranks"] == 8 and t["final_worlds"] == [8] and t["final_states_equal"], t
    assert t["first_step"] is not None and t["first_step"]["world"] == 7 and t["first_step"]["s"] > 0
    kinds = {e["kind"] for e in t["timeline"]}
    assert {"fault_injected", "epoch_formed", "step_done"} <= kinds, kinds


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
    assert "plain form" in d["ttr"]["error"] and d["time_to_recover_s"] is None
