#!/bin/bash
# Diagnostic for the round-2 GPU-tier failure (test_xgmi_sync_collectives_queue_behind_pending_async):
# runs the mixed-mode worker the round-2 way (no store barrier between iterations, 5 s deadline)
# several times and prints each rank's give-up record (round / phase / workgroup / peer /
# waited ms / reason) and host launch timestamps, so the cause can be read off the record.
set -eu -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/xgmi_diag
mkdir -p $out
for rep in 1 2 3 4; do
  port=$((29600 + rep))
  for r in 0 1; do
    RANK=$r WORLD_SIZE=2 PORT=$port OUT=$out/mixed.$rep XG_MODE=mixed XG_NOSYNC=1 XG_TIMEOUT=5 PYTHONPATH=. \
      timeout -k 10 120 python tests/helpers/xgmi_comm_worker.py > $out/mixed.$rep.log.$r 2>&1 &
  done
  wait || exit 1
  for r in 0 1; do echo "rep $rep rank $r: $(cat $out/mixed.$rep.$r)"; done
done
