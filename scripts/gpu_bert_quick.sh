#!/bin/bash
# BERT path check: attention + kernel numerics, then the BERT-large 1-GPU step.
set -u
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
mkdir -p gpurun_out/bq
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py tests/test_attention_gpu.py -m gpu > gpurun_out/bq/tests.log 2>&1 || { tail -40 gpurun_out/bq/tests.log; exit 1; }
tail -1 gpurun_out/bq/tests.log
timeout -k 10 300 python3 benchmarks/train_bench.py --model bert-large --batch 32 --steps 10 --warmup 3 > gpurun_out/bq/bert.log 2>&1 || { tail -20 gpurun_out/bq/bert.log; exit 1; }
grep -h '"metric"' gpurun_out/bq/bert.log
