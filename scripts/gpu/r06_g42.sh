set -u -o pipefail
# does a side thread's allocator growth stall the main thread?
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 240 python -u scripts/bg_grow_probe.py after-kill > gpurun_out/r06_bg_grow.json 2> gpurun_out/r06_bg_grow.err
rc=$?; cat gpurun_out/r06_bg_grow.json; tail -3 gpurun_out/r06_bg_grow.err; exit $rc
