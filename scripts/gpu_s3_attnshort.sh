#!/bin/bash
# Short-sequence attention forward (EDL_ATTN_SHORT): attention numerics tests, BERT-shape timings, BERT-large step A/B.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/ashort
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/ashort/pytest.log 2>&1 || { tail -30 gpurun_out/ashort/pytest.log; exit 1; }
tail -1 gpurun_out/ashort/pytest.log
for i in 1 2; do
  for sh in 1 0; do EDL_ATTN_SHORT=$sh timeout -k 10 120 python3 scripts/attn_time.py bert || exit 1; done
done
for i in 1 2; do
  for sh in 1 0; do
    EDL_ATTN_SHORT=$sh timeout -k 10 200 python3 benchmarks/train_bench.py --model bert-large --batch 32 --steps 20 \
      --warmup 3 > gpurun_out/ashort/b$sh.log 2>&1 || { tail -20 gpurun_out/ashort/b$sh.log; exit 1; }
    echo "bert EDL_ATTN_SHORT=$sh $(grep -h '"metric"' gpurun_out/ashort/b$sh.log | cut -c45-120)"
  done
done
