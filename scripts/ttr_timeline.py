"""Print the merged event timeline of a fault-drill run directory relative to the injected
fault (t_rel_s proc event fields).  usage: ttr_timeline.py <run_dir> [seconds_before]"""
import glob
import json
import os
import sys


def main():
    run = sys.argv[1]
    before = float(sys.argv[2]) if len(sys.argv) > 2 else 0.7
    ev = []
    for f in glob.glob(os.path.join(run, "events-*.jsonl")):
        for line in open(f):
            try:
                ev.append(json.loads(line))
            except ValueError:
                pass
    ev.sort(key=lambda e: e.get("mono", e["ts"]))
    t0 = next((e.get("mono", e["ts"]) for e in ev if e["kind"] == "fault_injected"), ev[0].get("mono", ev[0]["ts"]))
    for e in ev:
        t = e.get("mono", e["ts"]) - t0
        if t < -before:
            continue
        rest = {k: v for k, v in e.items() if k not in ("ts", "mono", "proc", "kind")}
        print(f"{t:8.3f} {e.get('proc', ''):10s} {e['kind']:16s} {json.dumps(rest)[:110]}")


if __name__ == "__main__":
    main()
