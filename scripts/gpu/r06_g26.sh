set -u -o pipefail
# Same-box step A/B: the curated GEMM selections vs + round-1's tuned lm_head solutions
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/r06_lmhead_tuning_ab.jsonl
: > $out
for i in 1 2 3; do
  for v in lmhead base; do
    f=easydl_amd/tuned/tunableop_gfx950_select.csv
    [ $v = lmhead ] && f=easydl_amd/tuned/tunableop_gfx950_select_lmhead.csv
    EDL_GEMM_TUNING_FILE=$f timeout -k 10 300 python -u bench.py --steps 8 --warmup 3 --ttr off \
      > gpurun_out/lt_${v}_${i}.json 2> gpurun_out/lt.err || exit 1
    python scripts/ab_line.py gpurun_out/lt_${v}_${i}.json "gemm_select=$v" $i >> $out || exit 1
    tail -1 $out
  done
done
