"""Print one A/B record (tree, run, value, ms_per_step) from a bench.py JSON output file."""
import json
import sys

if __name__ == "__main__":
    path, tree, run = sys.argv[1], sys.argv[2], int(sys.argv[3])
    d = json.loads(open(path).read().strip().splitlines()[-1])
    print(json.dumps({"tree": tree, "run": run, "value": d["value"], "ms_per_step": d["ms_per_step"]}))
