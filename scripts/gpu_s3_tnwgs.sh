#!/bin/bash
# TN split-M work target A/B (EDL_GEMM_TN_WGS = 256 one workgroup per CU, 512 two): BERT shapes + BERT-large step.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/tnwgs
for wgs in 256 512; do
  EDL_GEMM_TN_WGS=$wgs PYTHONPATH=$PWD timeout -k 10 200 python -u scripts/gemm_tn_bench.py bert_qkv bert_o bert_fc1 bert_fc2 \
    > gpurun_out/tnwgs/b$wgs.jsonl 2>&1 || { tail -5 gpurun_out/tnwgs/b$wgs.jsonl; exit 1; }
  grep shape gpurun_out/tnwgs/b$wgs.jsonl | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print('wgs=$wgs', d['shape'], d['tn_ms'], d['tn_pf'])"
done
for i in 1 2; do
  for wgs in 256 512; do
    EDL_GEMM_TN_WGS=$wgs timeout -k 10 200 python3 benchmarks/train_bench.py --model bert-large --batch 32 --steps 20 \
      --warmup 3 > gpurun_out/tnwgs/bert$wgs.log 2>&1 || { tail -20 gpurun_out/tnwgs/bert$wgs.log; exit 1; }
    echo "bert wgs=$wgs $(grep -h '"metric"' gpurun_out/tnwgs/bert$wgs.log | cut -c45-120)"
  done
done
