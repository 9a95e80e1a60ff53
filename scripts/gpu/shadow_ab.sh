#!/bin/bash
# Mid-step resume A/B at full Llama-3-8B width, 1 x 8 micro-batches of 8k tokens (where the gradient
# shadow fits beside a replacement's first step): the no-survivor drill with the shadow on (default)
# and off (EDL_GRAD_SHADOW=0), the worker killed once the GPU finished 4 of the 8 micro-batches.
# Each drill's JSON: TTR, resumed_mid_step, step time before the fault.
set -uo pipefail
out=gpurun_out/r05_${TAG:-shadow_ab}
mkdir -p $out
for mode in on off; do
  mkdir -p $out/$mode
  v=1; [ $mode = off ] && v=0
  EDL_BENCH_FAULT_SPEC="${FSPEC:-kill@step=4,index=0,point=microbatch,mb=3,wait=standby}" \
  EDL_GRAD_SHADOW=$v EDL_TTR_DIR=$out/$mode EDL_TTR_KEEP=1 \
    timeout -k 10 600 python -u bench.py --fault-inject --gpus 1 --fault-mode midstep --standby 1 \
    --fault-step 4 --mbs 1 --accum 8 --ckpt-interval 2 --steps 0 --warmup 0 > $out/$mode.json 2> $out/$mode.err
  rc=$?; echo "$mode rc=$rc"; cat $out/$mode.json; [ $rc -eq 0 ] || exit $rc
done
