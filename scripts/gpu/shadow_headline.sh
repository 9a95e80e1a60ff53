#!/bin/bash
# The headline drill (2 x 4 micro-batches) with the gradient shadow forced on: does the replacement's
# first step still fit beside it?  Kill 1: the driver's host-timed mid-step kill; kill 2: once the GPU
# finished micro-batch 1, plus half a micro-batch (inside micro-batch 2).
set -uo pipefail
out=gpurun_out/r05_${TAG:-shadow_headline}
mkdir -p $out
specs=("" "kill@step=4,index=0,point=microbatch,mb=1,after_ms=350,wait=standby")
[ -n "${ONLY:-}" ] && specs=("${specs[$ONLY]}")
i=0
for spec in "${specs[@]}"; do
  i=$((i+1)); mkdir -p $out/k$i
  EDL_BENCH_FAULT_SPEC="$spec" EDL_GRAD_SHADOW=${SHADOW:-force} EDL_TTR_DIR=$out/k$i EDL_TTR_KEEP=1 \
  EDL_FAULT_STEP_MS=2850 timeout -k 10 600 python -u bench.py --fault-inject --gpus 1 --fault-mode midstep \
    --standby 1 --fault-step 4 --mbs 2 --accum 4 --ckpt-interval 2 --steps 0 --warmup 0 > $out/k$i.json 2> $out/k$i.err
  rc=$?; echo "k$i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
