set -u -o pipefail
# three-failure soak WITHOUT the short standby warm-up (the configuration that crashed), HIP error log on
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
EDL_STANDBY_WARM_SHORT=0 AMD_LOG_LEVEL=1 TAG=r06_soak3_noshort bash scripts/gpu/soak_3fail.sh > gpurun_out/r06_soak_noshort.txt 2>&1
rc=$?; tail -c 300 gpurun_out/r06_soak_noshort.txt; exit $rc
