set -u -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r06_gpu_tier.log 2>&1
rc=$?; echo "gpu tier rc=$rc"; tail -5 gpurun_out/r06_gpu_tier.log; [ $rc -ge 124 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_smoke.log 2>&1
echo "smoke rc=$?"
