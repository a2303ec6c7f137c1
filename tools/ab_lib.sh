#!/bin/bash
# A/B of two builds of libmimi_hip.so on one box: bench.py with the in-tree library and with $BASE_LIB,
# alternated ROUNDS times (each run under its own time limit).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
BASE_LIB=${BASE_LIB:-tools/bin/libmimi_hip_base.so}
for i in $(seq 1 ${ROUNDS:-3}); do
  for v in new base; do
    if [ $v = base ]; then export MIMI_HIP_LIB=$R/$BASE_LIB; else unset MIMI_HIP_LIB; fi
    timeout -k 10 200 python bench.py --cpu-baseline-seconds 0 --no-f32-mode --steps 20 --warmup 5 ${BENCH_ARGS:-} > gpurun_out/ab_$v.json 2>/dev/null || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/ab_$v.json').read().strip().splitlines()[-1]); s=d.get('stages_ms_per_step',{}); keys='${KEYS:-}'.split(); print('$v', d['value'], d['ms_per_step'], {k: s[k] for k in sorted(s) if (k in keys if keys else k.startswith(('down','res')))})"
  done
done
