#!/bin/bash
# BERT packed-qkv attention reading q/k/v as row-strided slices (no split pass) vs the split
# path (EDL_ATTN_QKV_SPLIT=1): numerics, BERT-large step A/B, kernel profile of the new path.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/qkv_ab
timeout -k 10 400 python -u -m pytest tests/test_attention_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/qkv_ab/pytest.log 2>&1 || { tail -30 gpurun_out/qkv_ab/pytest.log; exit 1; }
tail -1 gpurun_out/qkv_ab/pytest.log
for i in 1 2 3; do
  timeout -k 10 200 python3 benchmarks/train_bench.py --model bert-large --batch 32 --steps 20 --warmup 3 \
    > gpurun_out/qkv_ab/new$i.log 2>&1 || { tail gpurun_out/qkv_ab/new$i.log; exit 1; }
  echo "bert strided: $(grep -h '"metric"' gpurun_out/qkv_ab/new$i.log | cut -c1-140)"
  EDL_ATTN_QKV_SPLIT=1 timeout -k 10 200 python3 benchmarks/train_bench.py --model bert-large --batch 32 --steps 20 \
    --warmup 3 > gpurun_out/qkv_ab/split$i.log 2>&1 || { tail gpurun_out/qkv_ab/split$i.log; exit 1; }
  echo "bert split:   $(grep -h '"metric"' gpurun_out/qkv_ab/split$i.log | cut -c1-140)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/qkv_ab/prof -o bert -- \
  python3 benchmarks/train_bench.py --model bert-large --batch 32 --steps 6 --warmup 2 > gpurun_out/qkv_ab/prof.log 2>&1 \
  || { tail gpurun_out/qkv_ab/prof.log; exit 1; }
echo "profile done"
