set -u -o pipefail
# three-failure soak with the standby HBM slab OFF (does the slab cause the rehome export failures?)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
EDL_STANDBY_SLAB=0 TAG=r06_soak3_noslab bash scripts/gpu/soak_3fail.sh > gpurun_out/r06_soak_noslab.txt 2>&1
rc=$?; tail -c 300 gpurun_out/r06_soak_noslab.txt; exit $rc
