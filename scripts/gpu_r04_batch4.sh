#!/bin/bash
# round 4, batch 4: gradient-dtype + side-stream tests (logs), the auto-plane drill long enough for the
# replacement to rejoin (cached policy adopted at world 3), the reference's example job (DeepFM CTR) on the
# GPU PS data plane with every role on GPU 0; results under gpurun_out/
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ttr_auto_rejoin
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_grad_dtype_gpu.py \
    "tests/test_kernels_gpu.py::test_bert_layer_residual_grad_slots_match_fp32" > gpurun_out/r04_grad_dtype_test.log 2>&1
EDL_TTR_KEEP=1 EDL_TTR_DIR=gpurun_out/ttr_auto_rejoin timeout -k 10 300 python -u bench.py --fault-inject --share-gpu \
    --gpus 3 --comm auto-gloo --model llama-tiny --seq 2048 --mbs 2 --accum 1 --steps 400 --warmup 2 --fault-step 4 \
    > gpurun_out/r04_drill_auto_gloo_rejoin.log 2>&1
timeout -k 10 400 python -m easydl_amd.cli submit examples/deepctr_ps_gpu.yaml --gpus 0,0,0,0,0,0,0 \
    --run-dir gpurun_out/deepctr_gpu --timeout 360 > gpurun_out/r04_deepctr_gpu.log 2>&1
