#!/bin/bash
# Stall breakdown of the attention kernels: where do waves spend their cycles?
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/pmc2
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_WAVES SQ_INSTS_MFMA"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  S=8192 ITERS=2 timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $P --output-format csv -d gpurun_out/pmc2/p$i -o a -- python3 scripts/attn_pmc.py > gpurun_out/pmc2/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
