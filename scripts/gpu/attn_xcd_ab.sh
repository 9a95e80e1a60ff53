#!/bin/bash
# dK/dV kernel with and without XCD-aware block renumbering (EDL_ATTN_DKDV_XCD) at the headline
# shape (B 2, S 8192, H 32, KV 8, causal): fwd / bwd time, min of 7, alternating runs; then the
# attention numerics tests with the renumbering on.
set -uo pipefail
out=gpurun_out/r05_attn_xcd; mkdir -p $out
for rep in 1 2; do
for x in 0 1; do
  EDL_ATTN_DKDV_XCD=$x timeout -k 10 200 python - > $out/xcd_${x}_$rep.json <<'PY' || exit 1
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
for _ in range(7):
    e[0].record(); flash_attention(q, k, v); e[1].record(); flash_attention(q, k, v).backward(do); e[2].record()
    torch.cuda.synchronize(); f = e[0].elapsed_time(e[1]); fb = e[1].elapsed_time(e[2]); ts.append((f, fb - f))
print(json.dumps({"xcd": os.environ["EDL_ATTN_DKDV_XCD"], "fwd_ms": round(min(t[0] for t in ts), 3), "bwd_ms": round(min(t[1] for t in ts), 3)}))
PY
  cat $out/xcd_${x}_$rep.json
done
done
EDL_ATTN_DKDV_XCD=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_attention_gpu.py > $out/pytest_xcd1.log 2>&1
rc=$?; tail -2 $out/pytest_xcd1.log; exit $rc
