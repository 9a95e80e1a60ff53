#!/bin/bash
# BERT-large 1-GPU step: fused GELU MLP + packed-qkv attention (default) vs both off
# (EDL_MLP_FUSED=0 EDL_ATTN_PACKED=0), interleaved on one box.
set -u
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
v() { python3 -c 'import json,sys; d=json.loads([l for l in sys.stdin if "metric" in l][-1]); print(d["value"], d["ms_per_step"])'; }
for i in 1 2 3; do
  a=$(timeout -k 10 300 python3 benchmarks/train_bench.py --model bert-large --batch 32 --steps 20 --warmup 3 2>&1 | v) || exit 1
  b=$(EDL_MLP_FUSED=0 EDL_ATTN_PACKED=0 timeout -k 10 300 python3 benchmarks/train_bench.py --model bert-large --batch 32 --steps 20 --warmup 3 2>&1 | v) || exit 1
  echo "round $i: on $a | off $b"
done
