#!/bin/bash
# End-to-end A/B of the curated TunableOp GEMM selections: 1-GPU Llama-3-8B
# bench with EDL_GEMM_TUNING=off / select, interleaved (off, select, off, select).
set -u
mkdir -p gpurun_out
for m in off select off select; do
  EDL_GEMM_TUNING=$m timeout -k 10 400 python bench.py --steps 8 --warmup 2 > gpurun_out/ab_$m.log 2>&1 || { tail -20 gpurun_out/ab_$m.log; exit 1; }
  grep -h '"metric"' gpurun_out/ab_$m.log \
    | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$m', d['value'], d['ms_per_step'], d['config'].get('gemm_tuning'))" \
    | tee -a gpurun_out/gemm_select_ab.txt
done
