set -u -o pipefail
# Same-box A/B of BERT-large (1 GPU, batch 32): round-5 final tree (ea107fc) vs head, alternating
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/r06_bert_tree_ab.jsonl
: > $out
for i in 1 2 3; do
  (cd abtmp/r05 && timeout -k 10 300 python benchmarks/train_bench.py --model bert-large --batch 32 --steps 10 \
    --warmup 3 > ../../gpurun_out/bert_r05_$i.json 2> ../../gpurun_out/bert_r05.err) || exit 1
  python scripts/ab_line.py gpurun_out/bert_r05_$i.json r05-ea107fc $i >> $out
  timeout -k 10 300 python benchmarks/train_bench.py --model bert-large --batch 32 --steps 10 --warmup 3 \
    > gpurun_out/bert_head_$i.json 2> gpurun_out/bert_head.err || exit 1
  python scripts/ab_line.py gpurun_out/bert_head_$i.json head $i >> $out
done
cat $out
