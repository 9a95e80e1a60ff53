set -u -o pipefail
# final-tree regression drills: world 8 on one GPU (kill -> 7 -> standby rejoin -> 8), then three
# successive failures at the headline config (replacement rehome, refill standby, HBM resume each time)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=r06final_world8 bash scripts/gpu/world8_drill.sh || exit 1
TAG=r06final_soak3 bash scripts/gpu/soak_3fail.sh || exit 1
