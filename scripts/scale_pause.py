"""Training pauses of the running world across world-size changes, from an event
timeline: last step at the old size -> first step at the new one (worker0's view).
Prints the first change (``pause``) and every change (``changes``)."""
import glob
import json
import os
import sys


def pause(run_dir: str) -> dict:
    ev = []
    for f in glob.glob(os.path.join(run_dir, "events-*.jsonl")):
        for ln in open(f):
            try:
                ev.append(json.loads(ln))
            except ValueError:
                pass
    ev.sort(key=lambda e: e["ts"])
    done = [e for e in ev if e["kind"] == "step_done" and e.get("proc") == "worker0"]
    warm = [e.get("s") for e in ev if e["kind"] == "prejoin_warmup"]
    out = []
    for a, b in zip(done, done[1:]):
        if b.get("world") != a.get("world"):
            steady = [y["ts"] - x["ts"] for x, y in zip(done, done[1:])
                      if x.get("world") == y.get("world") == b["world"]]
            out.append({"from_world": a["world"], "to_world": b["world"], "pause_s": round(b["ts"] - a["ts"], 3),
                        "steady_step_s_new_world": round(sorted(steady)[len(steady) // 2], 3) if steady else None})
    return dict(out[0], prejoin_warmup_s=warm, changes=out) if out else {}


if __name__ == "__main__":
    print(json.dumps(pause(sys.argv[1])))
