#!/bin/bash
# Attention forward variants at the Llama shape: default 32-queries-per-wave kernel vs EDL_ATTN_FWD=64.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for i in 1 2 3; do
  timeout -k 10 120 python3 scripts/attn_time.py || exit 1
  EDL_ATTN_FWD=64 timeout -k 10 120 python3 scripts/attn_time.py || exit 1
done
