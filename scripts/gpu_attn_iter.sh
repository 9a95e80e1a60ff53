#!/bin/bash
# attention kernel iteration: numerics, timing, PMC pass.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/attn
timeout -k 10 300 python3 -m pytest -q -x tests/test_attention_gpu.py > gpurun_out/attn/test.log 2>&1
rc=$?; tail -3 gpurun_out/attn/test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/attn_bench.py > gpurun_out/attn/bench.json 2> gpurun_out/attn/bench.err || exit $?
cat gpurun_out/attn/bench.json
EDL_ATTN_DKDV_OCC=2 timeout -k 10 300 python3 scripts/attn_bench.py > gpurun_out/attn/bench_occ2.json 2>> gpurun_out/attn/bench.err || exit $?
cat gpurun_out/attn/bench_occ2.json
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_MFMA"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc $P1 --output-format csv -d gpurun_out/attn/p1 -o attn -- python3 scripts/attn_pmc.py > gpurun_out/attn/p1.log 2>&1
echo "pmc rc=$?"
