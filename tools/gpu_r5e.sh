#!/bin/bash
# Round-5 session E: small batches with the fused q/k/v + attention forced (qkv_attn=2) vs auto (1)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5e
mkdir -p $O
for B in 1 4 8; do
  for F in 1 2 1 2; do
    timeout -k 10 200 python -u bench.py --batch $B --steps 40 --warmup 5 --cpu-baseline-seconds 0 --no-f32-mode --pmc-pass --option qkv_attn=$F --json-out $O/b${B}_qa$F.json > $O/b${B}_qa$F.log 2>&1 || exit 1
    python3 -c "import json; d=json.load(open('$O/b${B}_qa$F.json')); s=d.get('stages_ms_per_step',{}); print('B $B qkv_attn $F', d['value'], d['ms_per_step'], {k: s[k] for k in s if k in ('qkv','attention','qkv_attention','layernorm')})"
  done
done
