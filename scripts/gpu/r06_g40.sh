set -u -o pipefail
# three-failure soak with the HIP runtime's error log on (AMD_LOG_LEVEL=1: errors only), to see what
# precedes the third replacement's hipBLASLt initialisation failure
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
AMD_LOG_LEVEL=1 TAG=r06_soak3_log bash scripts/gpu/soak_3fail.sh > gpurun_out/r06_soak_log.txt 2>&1
rc=$?; tail -c 300 gpurun_out/r06_soak_log.txt; exit $rc
