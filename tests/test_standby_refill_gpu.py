"""A refill standby (spawned ~20 s after a takeover, while the replacement trains) warms up
only in a planned window between two steps: master ``warm_window_planned`` -> the worker's
``standby_warm_window`` (grant, pause, warm key) -> training goes on.  Llama-3-8B width, 2 layers,
on one GPU (VERDICT r4 Next #3)."""
import json
import os
import subprocess
import sys

import pytest

from easydl_amd.utils.events import read_events

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_refill_standby_warms_up_in_a_window(tmp_path):
    run_root = os.environ.get("EDL_TEST_KEEP_DIR") or str(tmp_path)
    env = dict(os.environ, EDL_TTR_DIR=run_root, EDL_TTR_KEEP="1")
    cmd = [sys.executable, "bench.py", "--fault-inject", "--gpus", "1", "--standby", "1", "--model", "llama3-8b",
           "--layers", "2", "--seq", "8192", "--mbs", "1", "--accum", "2", "--steps", "520", "--warmup", "0",
           "--fault-step", "4", "--fault-mode", "step_start"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=420)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert lines, r.stderr[-3000:]
    d = json.loads(lines[-1])
    assert d["operator_rc"] == 0 and d["replacement_from_standby"], d
    ev = read_events(d["run_dir"])
    planned = [e for e in ev if e["kind"] == "warm_window_planned"]
    windows = [e for e in ev if e["kind"] == "standby_warm_window"]
    assert planned and windows, [e["kind"] for e in ev][-40:]
    w = windows[0]
    assert w["warm"] and w["s"] < 30, w
    # the window sits between two committed steps of the replacement
    steps = sorted(e["step"] for e in ev if e["kind"] == "step_done" and e.get("epoch", 0) >= 2)
    assert steps and steps[0] <= w["step"] < steps[-1]
    print(json.dumps({"window": w, "planned": planned[0]}))
