"""Two failures of the same rank, both recovered from HBM (Llama-3-8B width, 2 layers, one GPU).

The first replacement adopted the dead worker's HBM over IPC and cannot export that memory
again, so it re-homes its state into its own allocations at a step boundary once the state is
settled (ElasticTrainer._maybe_rehome) and re-publishes it.  The refill standby warms up in a
planned window, adopts the re-published state when the replacement is killed in turn, and
resumes from HBM again instead of restoring /dev/shm.  Both kills land 40 ms into a step (its
forward in flight, the previous update done), as in the headline drill; a kill at a step's very
start can catch the previous update still running on the GPU, which the step marks then refuse."""
import json
import os
import subprocess
import sys

import pytest

from easydl_amd.utils.events import read_events

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_second_failure_resumes_from_hbm_again(tmp_path):
    run_root = os.environ.get("EDL_TEST_KEEP_DIR") or str(tmp_path)
    env = dict(os.environ, EDL_TTR_DIR=run_root, EDL_TTR_KEEP="1",
               EDL_BENCH_FAULT_SPEC="kill@step=4,index=0,gen=0,after_ms=40;"
                                    "kill@step=330,index=0,gen=1,after_ms=40,wait=standby")
    cmd = [sys.executable, "bench.py", "--fault-inject", "--gpus", "1", "--standby", "1", "--model", "llama3-8b",
           "--layers", "2", "--seq", "8192", "--mbs", "1", "--accum", "2", "--steps", "420", "--warmup", "0",
           "--fault-step", "4", "--fault-mode", "step_start"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=540)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert lines, r.stderr[-3000:]
    d = json.loads(lines[-1])
    assert d["operator_rc"] == 0, d
    ev = read_events(d["run_dir"])
    faults = [e for e in ev if e["kind"] == "fault_injected"]
    restored = [e for e in ev if e["kind"] == "restored"]
    rehomed = [e for e in ev if e["kind"] == "rehomed"]
    assert len(faults) == 2, [e["kind"] for e in ev][-30:]
    assert len(restored) == 2 and all(e["source"].startswith("hbm:") for e in restored), restored
    assert rehomed and rehomed[0]["step"] < faults[1]["step"], (rehomed, faults)
    print(json.dumps({"restored": restored, "rehomed": rehomed[0]}))
