#!/bin/bash
# Same-box A/B of the shipped TunableOp selection (EDL_GEMM_TUNING=select) against a full tuning file
# (FILE, default the round-5 full tuning of the training step), two alternating rounds of bench.py --child.
set -uo pipefail
out=gpurun_out/r05_tune_ab; mkdir -p $out
for i in 1 2; do
  for v in select r05; do
    if [ $v = select ]; then export EDL_GEMM_TUNING=select; unset EDL_GEMM_TUNING_FILE; else export EDL_GEMM_TUNING=use EDL_GEMM_TUNING_FILE=${FILE:-profiles/r05_tunableop_full_tuning.csv}; fi
    timeout -k 10 300 python -u bench.py --child --steps 8 --warmup 2 > $out/$v.$i.json 2> $out/$v.$i.err || exit 1
    echo "$v $i $(python -c "import json;d=json.load(open('$out/$v.$i.json'));print(d['value'], d['config']['gemm_tuning'])")"
  done
done
