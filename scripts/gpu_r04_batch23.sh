#!/bin/bash
# round 4, batch 23: configs 2 and 4 on the final tree (ResNet-50 and BERT-large 1 GPU, BERT-large async PS)
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u benchmarks/train_bench.py --model resnet50 --steps 20 --warmup 5 \
    > gpurun_out/r04_final_resnet50.log 2>&1
timeout -k 10 300 python -u benchmarks/train_bench.py --model bert-large --batch 32 --steps 20 --warmup 5 \
    > gpurun_out/r04_final_bert.log 2>&1
timeout -k 10 560 bash scripts/bert_ps_1gpu.sh > gpurun_out/r04_final_bert_ps.log 2>&1
