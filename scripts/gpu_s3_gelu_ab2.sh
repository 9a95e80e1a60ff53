#!/bin/bash
# GELU hardware-reciprocal A/B, second pass: 4 alternations, base first (abtmp/lib_gelu = before).
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/gelu2
BASE=$PWD/abtmp/lib_gelu
for i in 1 2 3 4; do
  EDL_LIBDIR=$BASE timeout -k 10 200 python3 benchmarks/train_bench.py --model bert-large --batch 32 --steps 30 \
    --warmup 3 > gpurun_out/gelu2/base$i.log 2>&1 || { tail gpurun_out/gelu2/base$i.log; exit 1; }
  echo "bert base: $(grep -h '"metric"' gpurun_out/gelu2/base$i.log | cut -c45-120)"
  timeout -k 10 200 python3 benchmarks/train_bench.py --model bert-large --batch 32 --steps 30 --warmup 3 \
    > gpurun_out/gelu2/new$i.log 2>&1 || { tail gpurun_out/gelu2/new$i.log; exit 1; }
  echo "bert new:  $(grep -h '"metric"' gpurun_out/gelu2/new$i.log | cut -c45-120)"
done
