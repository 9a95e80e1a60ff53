set -u -o pipefail
# TunableOp scratch-file probe (CPU-side crash at worst: a bad solution index in hipBLASLt)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
rm -f /tmp/edl_tunableop_scratch_*.csv
timeout -k 10 120 python -u scripts/tunableop_scratch_probe.py write > gpurun_out/r06_g38_write.log 2>&1
echo "write rc=$?"; cat gpurun_out/r06_g38_write.log | tail -30
echo "--- scratch after the write process exited:"; ls -la /tmp/edl_tunableop_scratch_*.csv; cat /tmp/edl_tunableop_scratch_*.csv
timeout -k 10 120 python -u scripts/tunableop_scratch_probe.py bogus > gpurun_out/r06_g38_bogus.log 2>&1
echo "bogus rc=$?"; cat gpurun_out/r06_g38_bogus.log | tail -30
