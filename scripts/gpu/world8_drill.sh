#!/bin/bash
# World-8 kill -> shrink -> rejoin on ONE GPU (VERDICT r4 Next #2c): 8 workers + 1 hot standby
# share the card over the default auto plane with gloo fallback (--comm auto-gloo), tiny model.
# The 8-GPU node form is the driver's; this rehearses its membership paths on real HIP contexts.
set -uo pipefail
out=gpurun_out/r05_${TAG:-world8}
mkdir -p $out/ttr
export EDL_TTR_DIR=$out/ttr EDL_TTR_KEEP=1 EDL_BENCH_UNTIL_REGROWN=1 EDL_BENCH_CAP=${CAP:-400} \
  EDL_FAULT_STEP_MS=${STEP_MS:-60}
timeout -k 10 ${LIMIT:-420} python -u bench.py --fault-inject --gpus 8 --share-gpu --comm auto-gloo --standby 1 \
  --model llama-tiny --seq ${SEQ:-2048} --mbs 1 --accum 1 --fault-mode midstep --fault-step ${FSTEP:-6} \
  --ckpt-interval 2 --steps 0 --warmup 0 "$@" > $out/drill.json 2> $out/drill.err
rc=$?; echo "world8 drill rc=$rc"; cat $out/drill.json; exit $rc
