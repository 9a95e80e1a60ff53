#!/bin/bash
# Side-stream transposes (EDL_TRANSPOSE_STREAM) for the NT weight gradients: bitwise test, Llama-3-8B step A/B.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/tstream
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "side_stream or swiglu or linear" -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/tstream/pytest.log 2>&1 || { tail -30 gpurun_out/tstream/pytest.log; exit 1; }
tail -1 gpurun_out/tstream/pytest.log
for i in 1 2; do
  for ts in 0 1; do
    EDL_TRANSPOSE_STREAM=$ts timeout -k 10 300 python3 bench.py --steps 6 --warmup 2 > gpurun_out/tstream/l$ts.log 2>&1 \
      || { tail -20 gpurun_out/tstream/l$ts.log; exit 1; }
    echo "llama EDL_TRANSPOSE_STREAM=$ts $(grep -h '"metric"' gpurun_out/tstream/l$ts.log | cut -c150-250)"
  done
done
