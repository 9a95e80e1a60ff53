#!/bin/bash
# round 4, batch 2: gradient-dtype tests, side-stream residual-grad test, sparse PS GPU path, the auto-plane
# kill->shrink->rejoin drill, config-5 shard sizing, the grad-dtype bench A/B; results under gpurun_out/
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ttr_auto
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
    tests/test_ps_sparse.py > gpurun_out/r04_b2_tests.log 2>&1
EDL_TTR_KEEP=1 EDL_TTR_DIR=gpurun_out/ttr_auto timeout -k 10 300 python -u bench.py --fault-inject --share-gpu \
    --gpus 3 --comm auto-gloo --model llama-tiny --seq 256 --mbs 1 --accum 1 --steps 8 --warmup 2 --fault-step 4 \
    > gpurun_out/r04_drill_auto_gloo.log 2>&1
for cfg in "--mbs 2 --accum 4 --recompute 1" "--mbs 1 --accum 4 --recompute 0" "--mbs 2 --accum 4 --recompute 0"; do
  timeout -k 10 300 python -u -m easydl_amd.trainer.tp_dryrun --model llama3-70b --tp 8 $cfg \
      --out gpurun_out/r04_tp_dryrun.jsonl >> gpurun_out/r04_tp_dryrun.log 2>&1
done
for gd in bf16 fp32; do
  timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --grad-dtype $gd --out gpurun_out/r04_bench_grad_$gd.json \
      > gpurun_out/r04_bench_grad_$gd.log 2>&1
done
