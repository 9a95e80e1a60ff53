#!/bin/bash
# Round 3: IPC lifetime test; TP=2 (2 ranks sharing one GPU, xGMI engine only) with the
# TP collectives overlapped vs blocking (2-layer Llama-3-70B, seq 4096).
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_xgmi_gpu.py -k "lifetime or abort" > gpurun_out/r03g_lifetime.log 2>&1
for ov in 1 0; do
  EDL_TP_OVERLAP=$ov timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --tp 2 --share-gpu --layers 2 \
    --model llama3-70b --seq 4096 --mbs 1 --accum 1 --steps 6 --warmup 2 --comm xgmi-only \
    --out gpurun_out/r03g_tp2_overlap${ov}.json > gpurun_out/r03g_tp2_overlap${ov}.log 2>&1
done
tail -3 gpurun_out/r03g_lifetime.log
