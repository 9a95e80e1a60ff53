#!/bin/bash
# The N=1 time-to-recover drill alone, at the headline config (args override), run dir kept.
set -uo pipefail
out=gpurun_out/r05_${TAG:-drill}
mkdir -p $out/ttr
export EDL_TTR_DIR=$out/ttr EDL_TTR_KEEP=1 EDL_FAULT_STEP_MS=${STEP_MS:-2850}
timeout -k 10 600 python -u bench.py --fault-inject --gpus 1 --fault-mode ${MODE:-midstep} --standby 1 \
  --fault-step ${FSTEP:-4} --mbs 2 --accum 4 --ckpt-interval 2 --steps 0 --warmup 0 "$@" > $out/drill.json 2> $out/drill.err
rc=$?; echo "drill rc=$rc"; cat $out/drill.json; exit $rc
