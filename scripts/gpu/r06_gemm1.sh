set -u -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
ARMS=${ARMS:-"v8:0:8,v8p:2:8,v8p_g4:2:4,v8p_g16:2:16"}
timeout -k 10 400 python -u scripts/gemm_nt_bench.py --arms $ARMS --rounds 4 \
  --only ${ONLY:-qkv.fwd,gate_up.fwd,down.fwd,gate_up.dgrad,qkv.wgrad,lm_head.fwd} > gpurun_out/${OUT:-r06_gemm_v8_b}.jsonl 2>&1
rc=$?; python scripts/gemm_arms_table.py gpurun_out/${OUT:-r06_gemm_v8_b}.jsonl; exit $rc
