set -u -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
EDL_ATTN_DKDV_PF=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu \
  tests/test_attention_gpu.py > gpurun_out/r06_g8_attn_pf_tests.log 2>&1
rc=$?; echo "pf tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  EDL_ATTN_DKDV_PF=0 timeout -k 10 120 python scripts/attn_ab_dkdv.py >> gpurun_out/r06_attn_dkdv_pf3_ab.jsonl || exit 1
  EDL_ATTN_DKDV_PF=1 timeout -k 10 120 python scripts/attn_ab_dkdv.py >> gpurun_out/r06_attn_dkdv_pf3_ab.jsonl || exit 1
done
cat gpurun_out/r06_attn_dkdv_pf3_ab.jsonl
for pf in 0 1; do
  EDL_ATTN_DKDV_PF=$pf AB_ITERS=3 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r06_attn_prof3_pf$pf -o run -- python3 scripts/attn_ab_dkdv.py > /dev/null 2>&1 || exit 1
done
echo done-all
