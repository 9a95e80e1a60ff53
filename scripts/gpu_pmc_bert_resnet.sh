#!/bin/bash
# rocprofv3 PMC passes (HBM bytes, MFMA / LDS activity) over the BERT and ResNet hot
# kernels driven by scripts/pmc_bert_resnet.py; one counter group per pass.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/pmc2
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"
P2="FETCH_SIZE GRBM_GUI_ACTIVE"
P3="WRITE_SIZE GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $P --output-format csv \
  -d gpurun_out/pmc2/p$i -o k -- python3 scripts/pmc_bert_resnet.py > gpurun_out/pmc2/p$i.log 2>&1
  rc=$?; echo "pmc pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/pmc2/p$i.log; exit $rc; }
done
