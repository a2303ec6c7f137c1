#!/bin/bash
# Round-5 session U: res1_stream as separate uniform / ragged instantiations vs HEAD (ab/libmimi_hip_r1s0.so, one kernel
# with run-time-branched ragged lookups): res1_stream tests, then B = 32 and YODAS2-style timing alternated
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r5u"
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_res1_stream.py > "$O/pytest.log" 2>&1
rc=$?; tail -2 "$O/pytest.log"; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export MIMI_HIP_LIB=$R/ab/libmimi_hip_r1s0.so; else unset MIMI_HIP_LIB; fi
    timeout -k 10 200 python -u bench.py --steps 20 --cpu-baseline-seconds 0 --no-f32-mode --pmc-pass --json-out $O/b32_${v}_$i.json > $O/b32_${v}_$i.log 2>&1 || { tail -5 $O/b32_${v}_$i.log; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b32_${v}_$i.json')); s=d['stages_ms_per_step']; print('b32 $v', d['value'], d['ms_per_step'], 'res1_s2', s.get('res1_s2'))"
    timeout -k 10 200 python -u bench.py --workload yodas2 --steps 6 --warmup 2 --cpu-baseline-seconds 0 --json-out $O/y_${v}_$i.json > $O/y_${v}_$i.log 2>&1 || { tail -5 $O/y_${v}_$i.log; exit 1; }
    python3 -c "import json; d=json.load(open('$O/y_${v}_$i.json')); s=d['stages_ms_per_step']; print('yodas2 $v', d['value'], d['ms_per_step'], 'res1_s2', s.get('res1_s2'))"
  done
done
