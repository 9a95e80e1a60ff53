#!/bin/bash
# BASELINE.json config 5: Llama-3-70B, TP=8 over the node's xGMI mesh, elastic
# DP x TP trainer, async in-memory snapshots.  One process per GPU (8 GPUs).
#   bash benchmarks/llama70b_tp8.sh [steps] [warmup]
# Per GPU: 8.8e9 parameters (bf16 weights 17.6 GB + fp32 master/m/v 106 GB +
# bf16 grads 17.6 GB) + activations of one 8k sequence (~50 GB) ~= 190 GB of 288.
set -eu
STEPS=${1:-5}
WARMUP=${2:-2}
export HSA_ENABLE_IPC_MODE_LEGACY=0
exec python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29533 \
  "$(dirname "$0")/../bench.py" --gpus 8 --tp 8 --model llama3-70b --seq 8192 --mbs 1 --accum 4 \
  --steps "$STEPS" --warmup "$WARMUP" --ckpt-interval 10
