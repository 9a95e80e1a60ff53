"""Print a compact table of scripts/gemm_nt_bench.py JSONL output (TF/s per arm)."""
import json
import sys

for line in open(sys.argv[1]):
    if not line.startswith("{"):
        print(line.rstrip()[:300])
        continue
    d = json.loads(line)
    arms = [k for k, v in d.items() if isinstance(v, dict) and "tflops" in v]
    print(d["shape"], " ".join(f"{k}={d[k]['tflops']}" + (f"({d[k].get('rel_err')})" if "rel_err" in d[k] else "")
                               for k in arms))
