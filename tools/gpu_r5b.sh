#!/bin/bash
# Round-5 session B: res1_stream parity + A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5b
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_res1_stream.py -k "8-240000 or ragged" > $O/pytest_res1_stream.log 2>&1
rc=$?; echo "res1_stream tests rc=$rc"; grep -E "PASS|FAIL|Error|assert" $O/pytest_res1_stream.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for F in 0 4 5 6 7 0 4 5 6 7; do
  timeout -k 10 200 python -u bench.py --steps 20 --cpu-baseline-seconds 0 --no-f32-mode --pmc-pass --option res1_stream=$F --json-out $O/ab_stream_$F.json > $O/ab_stream_$F.log 2>&1
  rc=$?
  python3 -c "import json,sys; d=json.load(open('$O/ab_stream_$F.json')); s=d['stages_ms_per_step']; print('res1_stream $F', d['value'], 'res1_s2', s.get('res1_s2'), 'res1_s3', s.get('res1_s3'))"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
