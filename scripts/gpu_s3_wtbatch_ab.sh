#!/bin/bash
# Cached W^T refreshed in one multi-tensor transpose launch per step (EDL_WT_BATCH=1) vs one
# launch per weight: numerics, BERT-large and Llama-3-8B step A/B, BERT kernel profile.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/wtb
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_attention_gpu.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/wtb/pytest.log 2>&1 || { tail -30 gpurun_out/wtb/pytest.log; exit 1; }
tail -1 gpurun_out/wtb/pytest.log
for i in 1 2 3; do
  for b in 1 0; do
    EDL_WT_BATCH=$b timeout -k 10 200 python3 benchmarks/train_bench.py --model bert-large --batch 32 --steps 20 \
      --warmup 3 > gpurun_out/wtb/bert$b.log 2>&1 || { tail gpurun_out/wtb/bert$b.log; exit 1; }
    echo "bert EDL_WT_BATCH=$b $(grep -h '"metric"' gpurun_out/wtb/bert$b.log | cut -c45-120)"
  done
done
for b in 1 0; do
  EDL_WT_BATCH=$b timeout -k 10 300 python3 bench.py --steps 6 --warmup 2 > gpurun_out/wtb/llama$b.log 2>&1 \
    || { tail gpurun_out/wtb/llama$b.log; exit 1; }
  echo "llama EDL_WT_BATCH=$b $(grep -h '"metric"' gpurun_out/wtb/llama$b.log | cut -c150-260)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/wtb/prof -o bert -- \
  python3 benchmarks/train_bench.py --model bert-large --batch 32 --steps 6 --warmup 2 > gpurun_out/wtb/prof.log 2>&1 \
  || { tail gpurun_out/wtb/prof.log; exit 1; }
echo "profile done"
