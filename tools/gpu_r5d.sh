#!/bin/bash
# Round-5 session D: the folded ELU scalings (stage 0 / stage 1): parity tests, then A/B against ab/libmimi_hip_base.so
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5d
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_stage0_fused.py tests/test_res1_form.py tests/test_gpu_parity.py -k "not chain_give_up" > $O/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/pytest.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $O/pytest.log | head; exit $rc; fi
for i in 1 2 3; do
  for v in new base; do
    if [ $v = base ]; then export MIMI_HIP_LIB=$PWD/ab/libmimi_hip_base.so; else unset MIMI_HIP_LIB; fi
    timeout -k 10 200 python -u bench.py --steps 20 --cpu-baseline-seconds 0 --no-f32-mode --pmc-pass --json-out $O/ab_${v}_$i.json > $O/ab_${v}_$i.log 2>&1 || exit 1
    python3 -c "import json; d=json.load(open('$O/ab_${v}_$i.json')); s=d['stages_ms_per_step']; print('$v', d['value'], 'res_down_s0', s.get('res_down_s0'), 'res_s1', s.get('res_s1'))"
  done
done
