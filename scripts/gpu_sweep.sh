#!/bin/bash
# attention kernel check + batch-shape sweep of the headline bench
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_attention_gpu.py -x -q -s > gpurun_out/attn_test.log 2>&1
rc=$?; echo "attn tests rc=$rc"; grep "\[attn\]" gpurun_out/attn_test.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python scripts/attn_bench.py > gpurun_out/attn_bench.log 2>&1; echo "attn bench rc=$?"; tail -1 gpurun_out/attn_bench.log
for args in "--mbs 2" "--accum 2" "--mbs 2 --accum 2"; do
  timeout -k 10 500 python bench.py --steps 6 --warmup 2 $args > gpurun_out/sweep.log 2>&1
  rc=$?; echo "bench $args rc=$rc"; tail -1 gpurun_out/sweep.log | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
done
