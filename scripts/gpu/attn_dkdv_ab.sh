#!/bin/bash
# dK/dV kernel variants at the headline shape (B 2, S 8192, H 32, KV 8): 64 keys/wave (default),
# 32 keys/wave at 1 and 2 waves per SIMD; attention fwd and bwd time, min of 5.
set -uo pipefail
out=gpurun_out/r05_attn_ab; mkdir -p $out
for v in "64 1" "32 1" "32 2"; do
  set -- $v
  EDL_ATTN_DKDV=$1 EDL_ATTN_DKDV_OCC=$2 timeout -k 10 200 python - > $out/dkdv_$1_$2.json <<'PY' || exit 1
import json, os, sys, torch
sys.path.insert(0, os.getcwd())
os.environ["EDL_ATTN"] = "hip"
from easydl_amd.ops.attention import flash_attention
dev = torch.device("cuda", 0)
B, S, H, KV = 2, 8192, 32, 8
q = torch.randn(B, S, H, 128, device=dev, dtype=torch.bfloat16).transpose(1, 2).requires_grad_()
k = torch.randn(B, S, KV, 128, device=dev, dtype=torch.bfloat16).transpose(1, 2).requires_grad_()
v = torch.randn(B, S, KV, 128, device=dev, dtype=torch.bfloat16).transpose(1, 2).requires_grad_()
o = flash_attention(q, k, v); do = torch.randn_like(o)
for _ in range(3): flash_attention(q, k, v).backward(do)
torch.cuda.synchronize()
e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
ts = []
for _ in range(5):
    e[0].record(); flash_attention(q, k, v); e[1].record(); flash_attention(q, k, v).backward(do); e[2].record()
    torch.cuda.synchronize(); f = e[0].elapsed_time(e[1]); fb = e[1].elapsed_time(e[2]); ts.append((f, fb - f))
print(json.dumps({"dkdv": os.environ["EDL_ATTN_DKDV"], "occ": os.environ["EDL_ATTN_DKDV_OCC"], "fwd_ms": round(min(t[0] for t in ts), 3), "bwd_ms": round(min(t[1] for t in ts), 3)}))
PY
  cat $out/dkdv_$1_$2.json
done
