#!/bin/bash
# A/B of library builds on one box: bench.py with each of $LIBS ("new" = the in-tree libmimi_hip.so, else
# ab/libmimi_hip_<name>.so (ab/ travels to the box; tools/bin does not)), alternated ROUNDS times, each run under its own time limit.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
for i in $(seq 1 ${ROUNDS:-2}); do
  for v in ${LIBS:-base}; do
    if [ $v = new ]; then unset MIMI_HIP_LIB; else export MIMI_HIP_LIB=$R/ab/libmimi_hip_$v.so; fi
    timeout -k 10 200 python bench.py --cpu-baseline-seconds 0 --no-f32-mode --steps ${STEPS:-20} --warmup 5 ${BENCH_ARGS:-} > gpurun_out/ab_$v.json 2>gpurun_out/ab_$v.err || { echo "bench $v failed"; tail -5 gpurun_out/ab_$v.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/ab_$v.json').read().strip().splitlines()[-1]); s=d.get('stages_ms_per_step',{}); keys='${KEYS:-}'.split(); print('$v', d['value'], d['ms_per_step'], {k: s[k] for k in sorted(s) if (k in keys if keys else True)})"
  done
done
