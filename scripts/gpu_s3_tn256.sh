#!/bin/bash
# 256 x 256 TN weight-gradient kernel: numerics, per-shape microbench (both TN kernels vs hipBLASLt NT
# + transposes), Llama-3-8B step with EDL_WGRAD_TN=1 (every weight on TN) vs the auto policy.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/tn256
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "tn or colsum" -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/tn256/pytest.log 2>&1 || { tail -30 gpurun_out/tn256/pytest.log; exit 1; }
tail -1 gpurun_out/tn256/pytest.log
PYTHONPATH=$PWD timeout -k 10 300 python -u scripts/gemm_tn_bench.py llama_qkv llama_o llama_gu llama_down \
  > gpurun_out/tn256/bench256.jsonl 2>&1 || { tail -5 gpurun_out/tn256/bench256.jsonl; exit 1; }
grep shape gpurun_out/tn256/bench256.jsonl
for tn in 1 auto; do
  EDL_WGRAD_TN=$tn timeout -k 10 300 python3 bench.py --steps 6 --warmup 2 > gpurun_out/tn256/llama_$tn.log 2>&1 \
    || { tail -20 gpurun_out/tn256/llama_$tn.log; exit 1; }
  echo "llama EDL_WGRAD_TN=$tn $(grep -h '"metric"' gpurun_out/tn256/llama_$tn.log | cut -c150-250)"
done
