#!/bin/bash
# Round-5 session I: stage-0 phase probes -- conv waves without MFMAs (S0F_DIAG 1), block waves without blocks (2)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5i
mkdir -p $O
for i in 1 2; do
  for v in new s0diag1 s0diag2; do
    if [ $v = new ]; then unset MIMI_HIP_LIB; else export MIMI_HIP_LIB=$PWD/ab/libmimi_hip_$v.so; fi
    timeout -k 10 200 python -u bench.py --steps 20 --cpu-baseline-seconds 0 --no-f32-mode --pmc-pass --json-out $O/${v}_$i.json > $O/${v}_$i.log 2>&1 || { tail -5 $O/${v}_$i.log; exit 1; }
    python3 -c "import json; d=json.load(open('$O/${v}_$i.json')); s=d['stages_ms_per_step']; print('$v', d['value'], 'res_down_s0', s.get('res_down_s0'), 'reruns', d.get('f16x3'))"
  done
done
