#!/bin/bash
# ResNet-50 1-GPU step with the BatchNorm backward savings on (default) vs off
# (EDL_BN_DIRECT_GRADS=0 EDL_BN_MASK_FROM_X=0), interleaved on one box; BN tests first.
set -u
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_batchnorm_gpu.py -m gpu 2>&1 | tail -1
EDL_BN_DIRECT_GRADS=0 EDL_BN_MASK_FROM_X=0 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_batchnorm_gpu.py -m gpu 2>&1 | tail -1
v() { python3 -c 'import json,sys; d=json.loads([l for l in sys.stdin if "metric" in l][-1]); print(d["value"], d["ms_per_step"])'; }
for i in 1 2 3; do
  a=$(timeout -k 10 300 python3 benchmarks/train_bench.py --model resnet50 --batch 256 --steps 30 --warmup 5 2>&1 | v) || exit 1
  b=$(EDL_BN_DIRECT_GRADS=0 EDL_BN_MASK_FROM_X=0 timeout -k 10 300 python3 benchmarks/train_bench.py --model resnet50 --batch 256 --steps 30 --warmup 5 2>&1 | v) || exit 1
  echo "round $i: on $a | off $b"
done
