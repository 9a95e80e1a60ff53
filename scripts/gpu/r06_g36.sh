set -u -o pipefail
# final tree, second run of each drill: three successive failures at the headline config, then world 8
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=r06_soak3_final2 bash scripts/gpu/soak_3fail.sh > gpurun_out/r06_soak_final2.txt 2>&1 || exit 1
TAG=r06final_world8c bash scripts/gpu/world8_drill.sh > gpurun_out/r06_world8c.txt 2>&1 || exit 1
echo done
