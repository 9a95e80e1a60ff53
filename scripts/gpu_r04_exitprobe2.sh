#!/bin/bash
# round 4: when does a SIGKILLed GPU process's KFD entry disappear, relative to its reaping?
# (scripts/exit_cost_probe.cpp, built on the CPU host); results in gpurun_out/r04_exit_probe2.txt
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
ls -la /sys/class/kfd/kfd/proc/ > gpurun_out/r04_exit_probe2.txt 2>&1 || true
for m in gpu_memcpy pin; do
  timeout -k 10 200 ./scripts/exit_cost_probe.bin $m 64 >> gpurun_out/r04_exit_probe2.txt 2>&1
done
