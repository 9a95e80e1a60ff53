#!/bin/bash
# Three successive failures of the only worker at the headline config (Llama-3-8B, 2 x 4 micro-batches of
# 8k tokens, snapshots every 2 steps, hot standby; each kill 40 % into a step once the spare is warm):
# every replacement re-homes its adopted state, a refill standby warms in a planned window, and the next
# failure resumes from HBM again.  Events kept under gpurun_out/r05_${TAG:-soak3}/.
set -uo pipefail
out=gpurun_out/r05_${TAG:-soak3}
mkdir -p $out
EDL_TTR_DIR=$out EDL_TTR_KEEP=1 \
EDL_BENCH_FAULT_SPEC="kill@step=4,index=0,gen=0,after_ms=1120,wait=standby;kill@step=14,index=0,gen=1,after_ms=1120,wait=standby;kill@step=24,index=0,gen=2,after_ms=1120,wait=standby" \
  timeout -k 10 700 python -u bench.py --fault-inject --gpus 1 --standby 1 --mbs 2 --accum 4 --ckpt-interval 2 \
  --steps ${STEPS:-34} --warmup 0 --fault-step 4 --fault-mode step_start > $out/soak.json 2> $out/soak.err
rc=$?; echo "soak rc=$rc"; tail -c 600 $out/soak.json; exit $rc
