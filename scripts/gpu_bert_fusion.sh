#!/bin/bash
# BERT fusions (GELU MLP kernels with transposed outputs, packed-qkv attention gradients):
# kernel + attention numerics, BERT-large step, a short Llama-3-8B step (shared attention
# kernels), then a rocprofv3 kernel trace of the BERT step.
set -u
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
mkdir -p gpurun_out/bf
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py tests/test_attention_gpu.py -m gpu > gpurun_out/bf/tests.log 2>&1 || { tail -40 gpurun_out/bf/tests.log; exit 1; }
tail -1 gpurun_out/bf/tests.log
timeout -k 10 300 python3 benchmarks/train_bench.py --model bert-large --batch 32 --steps 10 --warmup 3 > gpurun_out/bf/bert.log 2>&1 || { tail -20 gpurun_out/bf/bert.log; exit 1; }
grep -h '"metric"' gpurun_out/bf/bert.log
timeout -k 10 300 python3 bench.py --steps 4 --warmup 2 > gpurun_out/bf/llama.log 2>&1 || { tail -20 gpurun_out/bf/llama.log; exit 1; }
grep -h '"metric"' gpurun_out/bf/llama.log
bash scripts/bert_profile.sh && python3 scripts/step_busy.py gpurun_out/bertprof/bert_kernel_trace.csv > gpurun_out/bertprof/busy.txt
