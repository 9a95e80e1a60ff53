#!/bin/bash
# Round 3: IPC lifetime test, then TunableOp tuning of the BERT-large GEMM shapes and an
# A/B of the BERT-large 1-GPU step with the tuned file vs the shipped selection.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
mkdir -p gpurun_out/r03i
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_xgmi_gpu.py -k "outlives" > gpurun_out/r03i/lifetime.log 2>&1
tail -2 gpurun_out/r03i/lifetime.log
timeout -k 10 300 python3 benchmarks/train_bench.py --model bert-large --batch 32 --steps 10 --warmup 3 \
  > gpurun_out/r03i/bert_select.log 2>&1
EDL_GEMM_TUNING=tune EDL_GEMM_TUNING_FILE=$PWD/gpurun_out/r03i/tunableop_bert.csv timeout -k 10 600 \
  python3 benchmarks/train_bench.py --model bert-large --batch 32 --steps 2 --warmup 1 > gpurun_out/r03i/bert_tune.log 2>&1
EDL_GEMM_TUNING=use EDL_GEMM_TUNING_FILE=$PWD/gpurun_out/r03i/tunableop_bert.csv timeout -k 10 300 \
  python3 benchmarks/train_bench.py --model bert-large --batch 32 --steps 10 --warmup 3 > gpurun_out/r03i/bert_use.log 2>&1
EDL_GEMM_TUNING=off timeout -k 10 300 \
  python3 benchmarks/train_bench.py --model bert-large --batch 32 --steps 10 --warmup 3 > gpurun_out/r03i/bert_off.log 2>&1
grep -h '"metric"' gpurun_out/r03i/bert_*.log | cut -c1-200
timeout -k 10 600 python bench.py --steps 6 --warmup 2 --out gpurun_out/r03i/bench_groups_split.json > gpurun_out/r03i/bench.log 2>&1
tail -1 gpurun_out/r03i/bench.log | cut -c1-300
