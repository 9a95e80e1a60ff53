#!/bin/bash
# BERT-large: transposed-weight cache (EDL_WT_CACHE, NT-form input gradients) on vs off.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/wtc
for i in 1 2; do
  for wc in 1 0; do
    EDL_WT_CACHE=$wc timeout -k 10 200 python3 benchmarks/train_bench.py --model bert-large --batch 32 --steps 20 \
      --warmup 3 > gpurun_out/wtc/b$wc.log 2>&1 || { tail -20 gpurun_out/wtc/b$wc.log; exit 1; }
    echo "bert EDL_WT_CACHE=$wc $(grep -h '"metric"' gpurun_out/wtc/b$wc.log | cut -c45-120)"
  done
done
