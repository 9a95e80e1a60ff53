"""dK/dV kernel A/B at the Llama-3-8B training shape (B2 S8192 H32 KV8 D128 causal): forward and
backward times of easydl_amd's flash attention, one JSON line.  The variant is chosen by the
environment of the process (EDL_ATTN_DKDV_PF is read once per process by the kernel library)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scripts.attn_bench import run  # noqa: E402

if __name__ == "__main__":
    r = run("hip", B=int(os.environ.get("AB_B", 2)), iters=int(os.environ.get("AB_ITERS", 10)))
    r["dkdv_pf"] = os.environ.get("EDL_ATTN_DKDV_PF", "0")
    print(json.dumps(r))
