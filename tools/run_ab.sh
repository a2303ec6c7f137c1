#!/bin/bash
# A/B of engine knobs on the bench (each run under its own limit; stop at the first failure).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 300 python bench.py --cpu-baseline-seconds 0 > gpurun_out/ab_$i.log 2>&1 || { echo "run $i ($cfg) failed"; exit 1; }
  echo "run $i ($cfg): $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_$i.log | head -1)"
done
