#!/bin/bash
# Same-box A/B of two curated TunableOp files (EDL_GEMM_TUNING_FILE): A=$AB_A vs B=$AB_B.
set -u
mkdir -p gpurun_out
run() {  # name file
  EDL_GEMM_TUNING=select EDL_GEMM_TUNING_FILE=$2 timeout -k 10 400 python bench.py --steps 8 --warmup 2 > gpurun_out/ab2_$1.log 2>&1 || { tail -20 gpurun_out/ab2_$1.log; exit 1; }
  grep -h '"metric"' gpurun_out/ab2_$1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1', d['value'], d['ms_per_step'])" | tee -a gpurun_out/gemm_select_ab2.txt
}
for i in 1 2; do
  run A "${AB_A:?csv}"
  run B "${AB_B:-easydl_amd/tuned/tunableop_gfx950_select.csv}"
done
