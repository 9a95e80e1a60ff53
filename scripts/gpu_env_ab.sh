#!/bin/bash
# A/B of a runtime environment variable (default HIP_FORCE_DEV_KERNARG=1: kernel arguments
# in device memory) on the launch-heavy steps (ResNet-50, BERT-large) and the Llama step,
# interleaved on one box.  Usage: VAR=NAME VAL=value bash scripts/gpu_env_ab.sh
set -u
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
VAR=${VAR:-HIP_FORCE_DEV_KERNARG}; VAL=${VAL:-1}
mkdir -p gpurun_out/envab
v() { python3 -c 'import json,sys; d=json.loads([l for l in sys.stdin if "metric" in l][-1]); print(d["value"], d["ms_per_step"])'; }
for i in 1 2; do
  for on in 1 0; do
    if [ $on = 1 ]; then E="env $VAR=$VAL"; else E="env -u $VAR"; fi
    r=$($E timeout -k 10 300 python3 benchmarks/train_bench.py --model resnet50 --batch 256 --steps 20 --warmup 5 2>&1 | v) || exit 1
    b=$($E timeout -k 10 300 python3 benchmarks/train_bench.py --model bert-large --batch 32 --steps 20 --warmup 3 2>&1 | v) || exit 1
    echo "$VAR on=$on resnet50 $r bert $b"
  done
done
for on in 1 0; do
  if [ $on = 1 ]; then E="env $VAR=$VAL"; else E="env -u $VAR"; fi
  l=$($E timeout -k 10 300 python3 bench.py --steps 4 --warmup 2 2>&1 | v) || exit 1
  echo "$VAR on=$on llama $l"
done
