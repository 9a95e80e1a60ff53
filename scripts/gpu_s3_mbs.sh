#!/bin/bash
# Llama-3-8B sequences per micro-batch: 2 (default) vs 3 (4 micro-batches per step either way).
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/mbs
for i in 1 2; do
  for m in 2 3; do
    timeout -k 10 400 python3 bench.py --steps 6 --warmup 2 --mbs $m > gpurun_out/mbs/m$m.log 2>&1 \
      || { tail -20 gpurun_out/mbs/m$m.log; exit 1; }
    echo "mbs=$m $(grep -h '"metric"' gpurun_out/mbs/m$m.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["peak_mem_gb"])')"
  done
done
