#!/bin/bash
# Stall breakdown + instruction-cache behaviour of the two attention forward kernels.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/pmcf
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmcf/counters.txt 2>&1 || true
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_WAVES SQ_INST_CYCLES_VMEM_RD"
P3="SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P --output-format csv -d gpurun_out/pmcf/p$i -o a -- python3 scripts/attn_fwd_pmc.py > gpurun_out/pmcf/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; tail -2 gpurun_out/pmcf/p$i.log
done
exit 0
