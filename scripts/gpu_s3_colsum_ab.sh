#!/bin/bash
# Column-sum kernels (slab reduce with a per-call block width, bf16 partials with row lanes and
# 8 loads in flight): kernel numerics, then a
# BERT-large step A/B against the previous library (abtmp/lib_base) and a kernel profile.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/colsum_ab
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_batchnorm_gpu.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/colsum_ab/pytest.log 2>&1 || { tail -30 gpurun_out/colsum_ab/pytest.log; exit 1; }
tail -1 gpurun_out/colsum_ab/pytest.log
BASE=$PWD/abtmp/lib_base
for i in 1 2; do
  timeout -k 10 200 python3 benchmarks/train_bench.py --model bert-large --batch 32 --steps 20 --warmup 3 \
    > gpurun_out/colsum_ab/new$i.log 2>&1 || { tail gpurun_out/colsum_ab/new$i.log; exit 1; }
  echo "bert new: $(grep -h '"metric"' gpurun_out/colsum_ab/new$i.log | cut -c1-200)"
  EDL_LIBDIR=$BASE timeout -k 10 200 python3 benchmarks/train_bench.py --model bert-large --batch 32 --steps 20 \
    --warmup 3 > gpurun_out/colsum_ab/base$i.log 2>&1 || { tail gpurun_out/colsum_ab/base$i.log; exit 1; }
  echo "bert base: $(grep -h '"metric"' gpurun_out/colsum_ab/base$i.log | cut -c1-200)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/colsum_ab/prof -o bert -- python3 benchmarks/train_bench.py \
  --model bert-large --batch 32 --steps 6 --warmup 2 > gpurun_out/colsum_ab/prof.log 2>&1 || { tail gpurun_out/colsum_ab/prof.log; exit 1; }
find gpurun_out/colsum_ab/prof -name "*kernel_stats.csv" | head -1
