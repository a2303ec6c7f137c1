#!/bin/bash
# Round-5 session G: ragged res1_stream parity, and host-fed workloads: this build vs the round-4 build (ab/)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5g
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_res1_stream.py > $O/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2; do
  for v in new r4; do
    if [ $v = r4 ]; then export MIMI_HIP_LIB=$PWD/ab/libmimi_hip_r4.so; else unset MIMI_HIP_LIB; fi
    for w in mls yodas2; do
      timeout -k 10 200 python -u bench.py --workload $w --steps 3 --warmup 1 --cpu-baseline-seconds 0 --json-out $O/${w}_${v}_$i.json > $O/${w}_${v}_$i.log 2>&1 || { tail -5 $O/${w}_${v}_$i.log; exit 1; }
      python3 -c "import json; d=json.load(open('$O/${w}_${v}_$i.json')); s=d['stages_ms_per_step']; print('$w $v', d['value'], d['ms_per_step'], 'dev', round(sum(s.values()),3), 'res1_s2', s.get('res1_s2'))"
    done
  done
done
for i in 1 2; do
  for v in new geludiag; do
    if [ $v = geludiag ]; then export MIMI_HIP_LIB=$PWD/ab/libmimi_hip_geludiag.so; else unset MIMI_HIP_LIB; fi
    timeout -k 10 200 python -u bench.py --steps 20 --cpu-baseline-seconds 0 --no-f32-mode --pmc-pass --json-out $O/b32_${v}_$i.json > $O/b32_${v}_$i.log 2>&1 || { tail -5 $O/b32_${v}_$i.log; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b32_${v}_$i.json')); s=d['stages_ms_per_step']; print('b32 $v', d['value'], d['ms_per_step'], 'fc1', s.get('fc1'), 'fc2', s.get('fc2'))"
  done
done
