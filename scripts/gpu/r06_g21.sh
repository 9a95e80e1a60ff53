set -u -o pipefail
# Llama-3-8B headline step: optimizer-update overlap on (default) vs off, alternating on one box
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/r06_opt_overlap_ab.jsonl
: > $out
for i in 1 2 3; do
  for v in 1 0; do
    EDL_OPT_OVERLAP=$v timeout -k 10 300 python -u bench.py --steps 8 --warmup 3 --ttr off > gpurun_out/oo_${v}_${i}.json 2> gpurun_out/oo.err || exit 1
    python scripts/ab_line.py gpurun_out/oo_${v}_${i}.json "opt_overlap=$v" $i >> $out || exit 1
    tail -1 $out
  done
done
