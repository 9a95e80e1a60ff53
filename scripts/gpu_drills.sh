#!/bin/bash
# One-GPU drills: BASELINE config 4 (BERT-large async PS, 2 PS + 6 workers sharing the GPU)
# and the Llama kill -> shrink -> rejoin drill (4 ranks sharing the GPU over the xGMI engine).
set -u -o pipefail
mkdir -p gpurun_out/ttr
if [ "${DRILL_BERT:-1}" = 1 ]; then
  bash scripts/bert_ps_1gpu.sh > gpurun_out/r03_bert_ps.txt 2>&1
  echo "bert_ps rc=$?"
  tail -16 gpurun_out/r03_bert_ps.txt
fi
EDL_HANG_DUMP_S=45 EDL_TTR_KEEP=1 EDL_TTR_DIR=gpurun_out/ttr timeout -k 10 170 python bench.py --fault-inject --share-gpu --gpus 4 \
  --layers 4 --seq 4096 --mbs 1 --accum 1 --warmup 3 --steps 10 --ckpt-interval 2 --standby 1 \
  > gpurun_out/r03_ttr_rejoin.json 2> gpurun_out/r03_ttr_rejoin.err
echo "ttr rc=$?"
cat gpurun_out/r03_ttr_rejoin.json
timeout -k 10 300 python -u -m pytest tests/test_tp.py tests/test_ps_sparse.py -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r03_tp_ps_tests.log 2>&1
echo "tp/ps tests rc=$?"
tail -4 gpurun_out/r03_tp_ps_tests.log
timeout -k 10 300 python scripts/attn_variant_ab.py EDL_ATTN_DKDV_MFMA default builtin asmvgpr > gpurun_out/r03_attn_dkdv_mfma_ab.txt 2>&1
echo "attn ab rc=$?"
tail -4 gpurun_out/r03_attn_dkdv_mfma_ab.txt
