#!/bin/bash
# round 4, batch 12: world-1 steps without the per-step host drain vs with it (EDL_STEP_SYNC=1), ResNet-50 batch 256
# (~35 ms steps) and BERT-large; then the headline model on the final tree
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
for s in 0 1 0 1; do
  EDL_STEP_SYNC=$s timeout -k 10 300 python3 benchmarks/train_bench.py --model resnet50 --batch 256 --steps 30 \
      --warmup 5 >> gpurun_out/r04_resnet_sync_ab.log 2>&1
done
for s in 0 1; do
  EDL_STEP_SYNC=$s timeout -k 10 300 python3 benchmarks/train_bench.py --model bert-large --batch 32 --steps 20 --warmup 3 \
      >> gpurun_out/r04_bert_sync_ab.log 2>&1
done
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r04_bench_final.log 2>&1
# where the replacement's first step after a no-survivor restore goes (1.2 s vs 0.4 s steady)
mkdir -p gpurun_out/ttr_n1_r12
EDL_STEP_PHASES=1 EDL_TTR_KEEP=1 EDL_TTR_DIR=gpurun_out/ttr_n1_r12 timeout -k 10 500 python -u bench.py --fault-inject \
    --gpus 1 --mbs 1 --accum 1 --steps 10 --warmup 7 --fault-step 10 > gpurun_out/r04_ttr_n1_phases2.log 2>&1
