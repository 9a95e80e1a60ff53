set -u -o pipefail
# BERT-large: optimizer-update group size vs the next forward's wait (head tree), alternating
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/r06_bert_groups.jsonl
: > $out
for p in 1 2; do
  for g in 1900 256 64 off; do
    if [ $g = off ]; then envs="EDL_OPT_OVERLAP=0"; else envs="EDL_FLAT_GROUP_MAX_MB=$g"; fi
    env $envs timeout -k 10 300 python benchmarks/train_bench.py --model bert-large --batch 32 --steps 10 \
      --warmup 3 > gpurun_out/bg.json 2> gpurun_out/bg.err || { tail -5 gpurun_out/bg.err; exit 1; }
    python scripts/ab_line.py gpurun_out/bg.json "groups_mb=$g" $p >> $out
    tail -1 $out
  done
done
