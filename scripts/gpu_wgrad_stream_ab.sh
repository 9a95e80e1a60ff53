#!/bin/bash
# Weight-gradient GEMMs on a side stream (EDL_WGRAD_STREAM=1) vs all on the compute stream:
# kernel tests, then the 1-GPU Llama-3-8B step interleaved 1/0/1/0 on the same box.
set -u
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
mkdir -p gpurun_out/ws
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py tests/test_attention_gpu.py -m gpu > gpurun_out/ws/tests.log 2>&1 || { tail -40 gpurun_out/ws/tests.log; exit 1; }
tail -1 gpurun_out/ws/tests.log
for v in 1 0 1 0; do
  EDL_WGRAD_STREAM=$v timeout -k 10 300 python3 bench.py --steps 4 --warmup 2 > gpurun_out/ws/b$v.log 2>&1 || { tail -20 gpurun_out/ws/b$v.log; exit 1; }
  echo "wgrad_stream=$v $(grep -h '"metric"' gpurun_out/ws/b$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["peak_mem_gb"])')"
done
EDL_WGRAD_STREAM=1 timeout -k 10 300 python3 benchmarks/train_bench.py --model bert-large --batch 32 --steps 10 --warmup 3 2>&1 | grep -h '"metric"' | cut -c1-200
EDL_WGRAD_STREAM=0 timeout -k 10 300 python3 benchmarks/train_bench.py --model bert-large --batch 32 --steps 10 --warmup 3 2>&1 | grep -h '"metric"' | cut -c1-200
