#!/bin/bash
# Round 3: dK/dV kernel with the exps of P pipelined under the dP MFMA chain
# (EDL_ATTN_DKDV_PIPE=1) vs the current kernel: numerics + interleaved timing, then the
# attention GPU tests with the variant on.
set -euo pipefail
mkdir -p gpurun_out/r03l
timeout -k 10 300 python scripts/attn_variant_ab.py EDL_ATTN_DKDV_PIPE 0 1 > gpurun_out/r03l/ab.txt 2>&1
cat gpurun_out/r03l/ab.txt
EDL_ATTN_DKDV_PIPE=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_attention_gpu.py -m gpu > gpurun_out/r03l/tests.log 2>&1
tail -1 gpurun_out/r03l/tests.log
