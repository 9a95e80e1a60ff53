#!/bin/bash
# Session-3 validation on one MI355X: GPU tier + smoke + Llama bench + kernel stats (gpu_validate.sh),
# BERT-large throughput + kernel trace, BERT-large async PS config 4 (2 PS + 6 workers on one GPU).
set -u
bash scripts/gpu_validate.sh || exit 1
timeout -k 10 200 python3 benchmarks/train_bench.py --model bert-large --batch 32 --steps 20 --warmup 3 \
  > gpurun_out/bert.log 2>&1 || { tail -20 gpurun_out/bert.log; exit 1; }
grep -h '"metric"' gpurun_out/bert.log
bash scripts/bert_profile.sh || exit 1
bash scripts/bert_ps_1gpu.sh
for i in 1 2; do
  for h in 0 1; do
    EDL_BN_RES_HANDOFF=$h timeout -k 10 300 python3 benchmarks/train_bench.py --model resnet50 --batch 256 --steps 20 \
      --warmup 3 > gpurun_out/rn_h$h.log 2>&1 || { tail -20 gpurun_out/rn_h$h.log; exit 1; }
    echo "resnet EDL_BN_RES_HANDOFF=$h $(grep -h '"metric"' gpurun_out/rn_h$h.log | cut -c40-140)"
  done
done
