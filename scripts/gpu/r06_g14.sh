set -u -o pipefail
# Same-box step A/B of the pipelined dK/dV slice (EDL_ATTN_DKDV_PF, default on) against round 5's
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/r06_dkdv_step_ab.jsonl
: > $out
for i in 1 2 3; do
  for v in 1 0; do
    EDL_ATTN_DKDV_PF=$v timeout -k 10 300 python -u bench.py --steps 8 --warmup 3 --ttr off > gpurun_out/r06_dkdv_ab_${v}_${i}.json 2> gpurun_out/r06_dkdv_ab.err || exit 1
    python scripts/ab_line.py gpurun_out/r06_dkdv_ab_${v}_${i}.json "dkdv_pf=$v" $i >> $out || exit 1
  done
done
cat $out
