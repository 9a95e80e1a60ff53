#!/bin/bash
# Wide-input TN rule (EDL_WGRAD_TN_WIDE_J): mixed-form SwiGLU test, Llama-3-8B step with the rule on (8192) vs off.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/tnwide
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "swiglu or tn" -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/tnwide/pytest.log 2>&1 || { tail -30 gpurun_out/tnwide/pytest.log; exit 1; }
tail -1 gpurun_out/tnwide/pytest.log
for i in 1 2; do
  for wj in 1000000 8192; do
    EDL_WGRAD_TN_WIDE_J=$wj timeout -k 10 300 python3 bench.py --steps 6 --warmup 2 > gpurun_out/tnwide/l$wj.log 2>&1 \
      || { tail -20 gpurun_out/tnwide/l$wj.log; exit 1; }
    echo "llama EDL_WGRAD_TN_WIDE_J=$wj $(grep -h '"metric"' gpurun_out/tnwide/l$wj.log | cut -c150-230)"
  done
done
