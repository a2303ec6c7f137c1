#!/bin/bash
# Several bench.py configurations in one GPU session (each under its own time limit; stop on a crash).
#   TAG=r2a bash tools/bench_matrix.sh
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
TAG=${TAG:-mx}
OUT="gpurun_out/$TAG"
mkdir -p "$OUT"
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py --cpu-baseline-seconds 0 "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"
  local rc=$?
  echo "$name rc=$rc $(python -c "import json,sys; d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], {k: d.get(k) for k in ('f32_mode_value','pcie_inclusive_value')})" 2>/dev/null)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -5 "$OUT/$name.err"; exit $rc; fi
}
# MATRIX: "name:args;name:args;..."
MATRIX=${MATRIX:-"b1:--batch 1 --no-f32-mode;b4:--batch 4 --no-f32-mode;b64:--batch 64 --no-f32-mode;s20:--seconds 20 --no-f32-mode;s60:--seconds 60 --batch 8 --no-f32-mode;yodas2:--workload yodas2 --steps 6 --warmup 2;mls:--workload mls --steps 3 --warmup 1"}
IFS=';' read -ra SPECS <<< "$MATRIX"
for spec in "${SPECS[@]}"; do
  name=${spec%%:*}; args=${spec#*:}
  run "$name" $args
done
