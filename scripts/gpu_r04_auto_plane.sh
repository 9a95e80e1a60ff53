#!/bin/bash
# round 4: the default "auto" data plane on hardware (ranks sharing one GPU) + a kill->shrink->rejoin
# drill on it, the gradient-dtype tests, the side-stream residual-grad test; results under gpurun_out/
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ttr_auto
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_xgmi_gpu.py \
    -k "auto_plane or ddp_step_xgmi_only" > gpurun_out/r04_auto_plane_test.log 2>&1
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_grad_dtype_gpu.py \
    "tests/test_kernels_gpu.py::test_bert_layer_residual_grad_slots_match_fp32" > gpurun_out/r04_grad_dtype_test.log 2>&1
EDL_TTR_KEEP=1 EDL_TTR_DIR=gpurun_out/ttr_auto timeout -k 10 300 python -u bench.py --fault-inject --share-gpu \
    --gpus 3 --comm auto-gloo --model llama-tiny --seq 256 --mbs 1 --accum 1 --steps 8 --warmup 2 --fault-step 4 \
    > gpurun_out/r04_drill_auto_gloo.log 2>&1
# config-5 sizing: one Llama-3-70B TP=8 shard at full depth (80 layers), seq 8192, loopback TP group
for cfg in "--mbs 2 --accum 4 --recompute 1" "--mbs 1 --accum 4 --recompute 0" "--mbs 2 --accum 4 --recompute 0"; do
  timeout -k 10 300 python -u -m easydl_amd.trainer.tp_dryrun --model llama3-70b --tp 8 $cfg \
      --out gpurun_out/r04_tp_dryrun.jsonl >> gpurun_out/r04_tp_dryrun.log 2>&1
done
