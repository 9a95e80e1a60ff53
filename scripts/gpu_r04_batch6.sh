#!/bin/bash
# round 4, batch 6: checkpoint GPU tests (incl. staged snapshots into an adopted segment); no-survivor restore
# TTR with the restored segment adopted (no unmap on the recovery path), pinned vs pageable (staged) slots;
# steady-state snapshot cost of the two slot kinds on the headline model; the rejoin drill with the
# micro-batch / all-reduce split of each step (EDL_STEP_PHASES=1)
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ttr_n1_r6 gpurun_out/ttr_phases2
cat /sys/kernel/mm/transparent_hugepage/shmem_enabled /sys/kernel/mm/transparent_hugepage/enabled \
    > gpurun_out/r04_thp.txt 2>&1 || true
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_ckpt_gpu.py \
    > gpurun_out/r04_b6_ckpt_tests.log 2>&1
EDL_TTR_KEEP=1 EDL_TTR_DIR=gpurun_out/ttr_n1_r6 timeout -k 10 400 python -u bench.py --fault-inject --gpus 1 \
    --mbs 1 --accum 1 --steps 4 --warmup 3 --fault-step 4 > gpurun_out/r04_ttr_n1_adopt_pin1.log 2>&1
EDL_SNAPSHOT_PIN=0 EDL_TTR_KEEP=1 EDL_TTR_DIR=gpurun_out/ttr_n1_r6 timeout -k 10 400 python -u bench.py \
    --fault-inject --gpus 1 --mbs 1 --accum 1 --steps 4 --warmup 3 --fault-step 4 \
    > gpurun_out/r04_ttr_n1_adopt_pin0.log 2>&1
EDL_SNAPSHOT_PIN=1 timeout -k 10 300 python -u bench.py --steps 8 --warmup 3 --ckpt-interval 2 \
    > gpurun_out/r04_bench_ckpt_pin1.log 2>&1
EDL_SNAPSHOT_PIN=0 timeout -k 10 300 python -u bench.py --steps 8 --warmup 3 --ckpt-interval 2 \
    > gpurun_out/r04_bench_ckpt_pin0.log 2>&1
EDL_STEP_PHASES=1 EDL_TTR_KEEP=1 EDL_TTR_DIR=gpurun_out/ttr_phases2 timeout -k 10 300 python -u bench.py \
    --fault-inject --share-gpu --gpus 3 --comm auto-gloo --model llama-tiny --seq 2048 --mbs 2 --accum 1 \
    --steps 400 --warmup 2 --fault-step 4 > gpurun_out/r04_drill_phases2.log 2>&1
