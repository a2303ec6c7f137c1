#!/bin/bash
# A/B of engine knobs on the bench: each argument is an env assignment list (e.g. "MIMI_X=1"), run in turn,
# ROUNDS times; prints audio-s/s, ms per step and the stages named in $STAGES (each run under its own limit;
# stops at the first failure).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
i=0
for r in $(seq 1 ${ROUNDS:-1}); do
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 300 python bench.py --cpu-baseline-seconds 0 --no-f32-mode --steps 20 --warmup 5 ${BENCH_ARGS:-} > gpurun_out/ab_$i.log 2>&1 || { echo "run $i ($cfg) failed"; tail -5 gpurun_out/ab_$i.log; exit 1; }
  python - "$cfg" gpurun_out/ab_$i.log <<'PY'
import json, os, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
st = d.get("stages_ms_per_step", {})
keys = os.environ.get("STAGES", "").split(",")
print(sys.argv[1], d["value"], d["ms_per_step"], {k: st[k] for k in keys if k in st})
PY
done
done
