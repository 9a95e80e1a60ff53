#!/bin/bash
# 256 x 256 TN kernel with row splits for BERT-size weights vs the 128 x 256 split kernel (EDL_GEMM_TN256).
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/tn256s
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "tn or colsum or gelu or bert" -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/tn256s/pytest.log 2>&1 || { tail -30 gpurun_out/tn256s/pytest.log; exit 1; }
tail -1 gpurun_out/tn256s/pytest.log
for m in 0 1; do
  EDL_GEMM_TN256=$m PYTHONPATH=$PWD timeout -k 10 200 python -u scripts/gemm_tn_bench.py bert_qkv bert_o bert_fc1 bert_fc2 \
    > gpurun_out/tn256s/b$m.jsonl 2>&1 || { tail -5 gpurun_out/tn256s/b$m.jsonl; exit 1; }
  grep shape gpurun_out/tn256s/b$m.jsonl | cut -c1-120 | sed "s/^/tn256=$m /"
done
for i in 1 2; do
  for m in 0 1; do
    EDL_GEMM_TN256=$m timeout -k 10 200 python3 benchmarks/train_bench.py --model bert-large --batch 32 --steps 20 \
      --warmup 3 > gpurun_out/tn256s/bert$m.log 2>&1 || { tail -20 gpurun_out/tn256s/bert$m.log; exit 1; }
    echo "bert tn256=$m $(grep -h '"metric"' gpurun_out/tn256s/bert$m.log | cut -c45-120)"
  done
done
