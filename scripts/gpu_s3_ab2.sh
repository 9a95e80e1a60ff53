#!/bin/bash
# Session 3: TN weight-gradient kernel numerics + per-shape microbench, then whole-step A/Bs:
# BERT-large (EDL_WGRAD_TN x EDL_RESGRAD), Llama-3-8B (EDL_WGRAD_TN), ResNet-50 MIOpen solvers.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/ab2
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "tn or colsum or gelu or bert or swiglu" -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/ab2/pytest.log 2>&1 || { tail -40 gpurun_out/ab2/pytest.log; exit 1; }
tail -1 gpurun_out/ab2/pytest.log
PYTHONPATH=$PWD timeout -k 10 300 python -u scripts/gemm_tn_bench.py > gpurun_out/ab2/gemm_tn_bench.jsonl 2>&1 || { tail -20 gpurun_out/ab2/gemm_tn_bench.jsonl; exit 1; }
cat gpurun_out/ab2/gemm_tn_bench.jsonl
bert() {  # $1 = label; env set by caller
  timeout -k 10 200 python3 benchmarks/train_bench.py --model bert-large --batch 32 --steps 20 --warmup 3 > gpurun_out/ab2/bert_$1.log 2>&1 || { tail -20 gpurun_out/ab2/bert_$1.log; return 1; }
  echo "bert $1 $(grep -h '"metric"' gpurun_out/ab2/bert_$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
for i in 1 2; do
  EDL_WGRAD_TN=0 EDL_RESGRAD=0 bert tn0_rg0_$i || exit 1
  EDL_WGRAD_TN=1 EDL_RESGRAD=0 bert tn1_rg0_$i || exit 1
  EDL_WGRAD_TN=1 EDL_RESGRAD=1 bert tn1_rg1_$i || exit 1
done
for tn in 0 1; do
  EDL_WGRAD_TN=$tn timeout -k 10 300 python3 bench.py --steps 6 --warmup 2 > gpurun_out/ab2/llama_tn$tn.log 2>&1 || { tail -20 gpurun_out/ab2/llama_tn$tn.log; exit 1; }
  echo "llama tn=$tn $(grep -h '"metric"' gpurun_out/ab2/llama_tn$tn.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["peak_mem_gb"])')"
done
