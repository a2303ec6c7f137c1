#!/bin/bash
# Round-5 session A: the RVQ-chain give-up tests, the concurrency determinism probe, the headline bench, and the
# ROLE_RES1P tile A/B (res1p_form).  Every GPU step under its own limit; stop at the first crash / timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5a
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "chain" > $O/pytest_chain.log 2>&1
rc=$?; echo "chain tests rc=$rc"; tail -4 $O/pytest_chain.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 500 python -u tools/det_concurrent.py 20 > $O/det.log 2>&1
rc=$?; echo "det rc=$rc"; grep -E "mismatch|TOTAL|differ" $O/det.log | tail -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --json-out $O/bench.json > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 600 $O/bench.json
if [ $rc -ne 0 ]; then exit $rc; fi
for F in 0 1 2 3 4 5 6 7; do
  timeout -k 10 200 python -u bench.py --steps 20 --cpu-baseline-seconds 0 --no-f32-mode --pmc-pass --option res1p_form=$F --json-out $O/ab_res1p_$F.json > $O/ab_res1p_$F.log 2>&1
  rc=$?
  python3 -c "import json,sys; d=json.load(open('$O/ab_res1p_$F.json')); s=d['stages_ms_per_step']; print('res1p_form $F', d['value'], 'res1_s2', s.get('res1_s2'), 'res1_s3', s.get('res1_s3'))"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
