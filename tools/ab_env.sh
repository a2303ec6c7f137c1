#!/bin/bash
# A/B of env-selected variants on one box: bench.py per value of $VAR in $VALS, ROUNDS times each (own time limits)
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out
for i in $(seq 1 ${ROUNDS:-2}); do
  for v in ${VALS}; do
    env "$VAR=$v" timeout -k 10 200 python bench.py --cpu-baseline-seconds 0 --no-f32-mode --steps ${STEPS:-40} --warmup 10 ${BENCH_ARGS:-} > gpurun_out/ab_$v.json 2>/dev/null || { echo "bench $v failed"; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/ab_$v.json').read().strip().splitlines()[-1]); s=d.get('stages_ms_per_step',{}); keys='${KEYS:-qkv o_proj fc1 fc2 final downsample input_proj res3_s2 res3_s3}'.split(); print('$VAR=$v', d['value'], d['ms_per_step'], {k: s[k] for k in sorted(s) if k in keys})"
  done
done
