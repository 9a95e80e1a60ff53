#!/bin/bash
# rocprofv3 PMC passes over a kernel driver script (default: the hand-written hot kernels,
# scripts/pmc_kernels.py; attention: DRIVER=scripts/attn_pmc.py).  One counter group per pass,
# never mixed with tracing domains; each pass under its own kill timeout.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
out=gpurun_out/${TAG:-pmc}
mkdir -p $out
DRIVER=${DRIVER:-scripts/pmc_kernels.py}
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"
P2="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
P3="FETCH_SIZE GRBM_GUI_ACTIVE"
P4="WRITE_SIZE GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -s KILL ${PASS_S:-240} rocprofv3 --kernel-trace --pmc $P --output-format csv \
    -d $out/p$i -o k -- python3 $DRIVER > $out/p$i.log 2>&1
  rc=$?; echo "pmc pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
