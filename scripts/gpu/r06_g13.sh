set -u -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_gemm_nt_gpu.py > gpurun_out/r06_g13_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/r06_g13_tests.log | head -20; [ $rc -ne 0 ] && exit $rc
# same-box A/B of the step: nt8 dgrad routed (head) vs hipBLASLt, alternating
for i in 1 2 3; do
  for v in 1 0; do
    EDL_GEMM_NT8_DGRAD=$v timeout -k 10 300 python -u bench.py --steps 8 --warmup 3 --ttr off > gpurun_out/r06_nt8_ab_${v}_${i}.json 2> gpurun_out/r06_nt8_ab.err || exit 1
    python scripts/ab_line.py gpurun_out/r06_nt8_ab_${v}_${i}.json "nt8_dgrad=$v" $i >> gpurun_out/r06_nt8_step_ab.jsonl || exit 1
  done
done
cat gpurun_out/r06_nt8_step_ab.jsonl
