set -u -o pipefail
# three-failure soak on the final tree (seventh run)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=r06_soak3_g bash scripts/gpu/soak_3fail.sh > gpurun_out/r06_soak_g.txt 2>&1
rc=$?; tail -c 300 gpurun_out/r06_soak_g.txt; exit $rc
