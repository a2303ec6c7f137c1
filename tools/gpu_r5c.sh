#!/bin/bash
# Round-5 session C: stage-0 ZIMG form parity + A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5c
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_stage0_fused.py > $O/pytest_s0.log 2>&1
rc=$?; echo "stage0 tests rc=$rc"; grep -E "PASS|FAIL|Error|assert" $O/pytest_s0.log | head -20
if [ $rc -ne 0 ]; then exit $rc; fi
for F in 1 2 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --cpu-baseline-seconds 0 --no-f32-mode --pmc-pass --option stage0_fused=$F --json-out $O/ab_s0_$F.json > $O/ab_s0_$F.log 2>&1
  rc=$?
  python3 -c "import json,sys; d=json.load(open('$O/ab_s0_$F.json')); s=d['stages_ms_per_step']; print('stage0_fused $F', d['value'], 'res_down_s0', s.get('res_down_s0'))"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
