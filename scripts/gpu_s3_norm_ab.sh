#!/bin/bash
# Norm forward with one wave per row for rows <= 2048 wide (EDL_NORM_WAVE_ROWS): numerics, BERT-large
# A/B against one block per row (EDL_NORM_WAVE_ROWS=0), kernel profile.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/norm
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_attention_gpu.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/norm/pytest.log 2>&1 || { tail -30 gpurun_out/norm/pytest.log; exit 1; }
tail -1 gpurun_out/norm/pytest.log
for i in 1 2; do
  for m in 0 1; do
    EDL_NORM_WAVE_ROWS=$m timeout -k 10 200 python3 benchmarks/train_bench.py --model bert-large --batch 32 --steps 30 \
      --warmup 3 > gpurun_out/norm/b$m.log 2>&1 || { tail gpurun_out/norm/b$m.log; exit 1; }
    echo "bert EDL_NORM_WAVE_ROWS=$m $(grep -h '"metric"' gpurun_out/norm/b$m.log | cut -c45-120)"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/norm/prof -o bert -- \
  python3 benchmarks/train_bench.py --model bert-large --batch 32 --steps 6 --warmup 2 > gpurun_out/norm/prof.log 2>&1 \
  || { tail gpurun_out/norm/prof.log; exit 1; }
echo "profile done"
