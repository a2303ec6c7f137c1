#!/bin/bash
# Round-5 session Y: MimiEncoder's pipeline on 2 engines (concurrency 2: consecutive batches on two streams) vs 1 --
# the equality test, then YODAS2- and MLS-style host-fed timing alternated
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r5y"
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "pipeline_engines or chunks_equals or thread" > "$O/pytest.log" 2>&1
rc=$?; tail -2 "$O/pytest.log"; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for c in 2 1; do
    timeout -k 10 300 python -u bench.py --workload yodas2 --steps 12 --warmup 4 --cpu-baseline-seconds 0 --concurrency $c --json-out $O/y_c${c}_$i.json > $O/y_c${c}_$i.log 2>&1 || { tail -5 $O/y_c${c}_$i.log; exit 1; }
    python3 -c "import json; d=json.load(open('$O/y_c${c}_$i.json')); print('yodas2 c$c', d['value'], d['ms_per_step'])"
    timeout -k 10 300 python -u bench.py --workload mls --steps 8 --warmup 4 --cpu-baseline-seconds 0 --concurrency $c --json-out $O/m_c${c}_$i.json > $O/m_c${c}_$i.log 2>&1 || { tail -5 $O/m_c${c}_$i.log; exit 1; }
    python3 -c "import json; d=json.load(open('$O/m_c${c}_$i.json')); print('mls c$c', d['value'], d['ms_per_step'])"
  done
done
