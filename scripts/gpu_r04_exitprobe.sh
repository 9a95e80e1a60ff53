#!/bin/bash
# round 4: teardown time of a SIGKILLed process by how it mapped a 64 GiB snapshot segment
# (scripts/exit_cost_probe.cpp; built on the CPU host); results in gpurun_out/r04_exit_probe.txt
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
for m in none populate_write memcpy pin populate_write_unmap; do
  timeout -k 10 200 ./scripts/exit_cost_probe.bin $m 64 >> gpurun_out/r04_exit_probe.txt 2>&1
done
