#!/bin/bash
# rocprofv3 PMC passes over the hand-written hot kernels (one pass per counter
# group; no tracing domains mixed with --pmc), then a kernel + memory-copy trace
# of a bench run with in-memory snapshots every step (D2H overlap evidence).
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/pmc
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"
P2="FETCH_SIZE GRBM_GUI_ACTIVE"
P3="WRITE_SIZE GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $P --output-format csv \
  -d gpurun_out/pmc/p$i -o k -- python3 scripts/pmc_kernels.py > gpurun_out/pmc/p$i.log 2>&1
  rc=$?; echo "pmc pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
  -d gpurun_out/pmc/ckpt -o bench -- python3 bench.py --steps 3 --warmup 1 --ckpt-interval 1 > gpurun_out/pmc/ckpt.log 2>&1
rc=$?; echo "ckpt trace rc=$rc"; grep metric gpurun_out/pmc/ckpt.log | tail -1
exit $rc
