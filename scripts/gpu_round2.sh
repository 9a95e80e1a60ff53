#!/bin/bash
# GPU tests, then the bench without and with in-memory snapshots (every 2 steps),
# then the attention stall-breakdown PMC passes.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 6 --warmup 2 > gpurun_out/bench_plain.log 2>&1 || exit $?
grep -h metric gpurun_out/bench_plain.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('plain', d['value'], d['ms_per_step'])"
timeout -k 10 400 python bench.py --steps 6 --warmup 2 --ckpt-interval 2 > gpurun_out/bench_ckpt2.log 2>&1 || exit $?
grep -h metric gpurun_out/bench_ckpt2.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('ckpt2', d['value'], d['ms_per_step'], d['ckpt'])"
bash scripts/gpu_pmc_attn2.sh
