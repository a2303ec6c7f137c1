#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in old d0 d1 d3 d4; do
  for bt in "32 250" "1 250"; do
    timeout -k 10 60 tools/bin/attn_check_$v $bt > gpurun_out/ac.log 2>&1 || { echo "attn_check_$v $bt failed"; cat gpurun_out/ac.log; exit 2; }
    echo "$v $bt: $(grep 'attention_t256_h16 ' gpurun_out/ac.log)"
  done
done
