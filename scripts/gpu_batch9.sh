#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_attention_gpu.py -x -q -s > gpurun_out/attn_test.log 2>&1
rc=$?; echo "attn tests rc=$rc"; grep -E "\[attn\]|passed|failed" gpurun_out/attn_test.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python scripts/attn_bench.py > gpurun_out/attn_bench.log 2>&1; echo "attn bench rc=$?"; tail -1 gpurun_out/attn_bench.log
timeout -k 10 400 python benchmarks/train_bench.py --model resnet50 --batch 256 > gpurun_out/resnet.log 2>&1; rc=$?; echo "resnet rc=$rc"; tail -1 gpurun_out/resnet.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python benchmarks/train_bench.py --model bert-large --batch 32 --seq 512 > gpurun_out/bert.log 2>&1; rc=$?; echo "bert rc=$rc"; tail -1 gpurun_out/bert.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 500 python bench.py --steps 6 --warmup 2 > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-300
