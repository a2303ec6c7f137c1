#!/bin/bash
# Round-5 session V: fc1's GELU with the branch-free erff replica (bitwise erff, tools/erf_check.hip) vs HEAD
# (ab/libmimi_hip_erf0.so): codes bitwise (tools/cmp_codes.py), then B = 32 and batch-1 timing alternated
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r5v"
mkdir -p "$O"
cd "$R"
timeout -k 10 200 python3 tools/lib_codes.py r5v_new > $O/codes_new.log 2>&1 || { tail -5 $O/codes_new.log; exit 1; }
MIMI_HIP_LIB=$R/ab/libmimi_hip_erf0.so timeout -k 10 200 python3 tools/lib_codes.py r5v_old > $O/codes_old.log 2>&1 || { tail -5 $O/codes_old.log; exit 1; }
python3 tools/cmp_codes.py r5v_old r5v_new || exit 1
for i in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export MIMI_HIP_LIB=$R/ab/libmimi_hip_erf0.so; else unset MIMI_HIP_LIB; fi
    timeout -k 10 200 python -u bench.py --steps 20 --cpu-baseline-seconds 0 --no-f32-mode --pmc-pass --json-out $O/b32_${v}_$i.json > $O/b32_${v}_$i.log 2>&1 || { tail -5 $O/b32_${v}_$i.log; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b32_${v}_$i.json')); s=d['stages_ms_per_step']; print('b32 $v', d['value'], d['ms_per_step'], 'fc1', s.get('fc1'))"
    timeout -k 10 200 python -u bench.py --batch 1 --steps 30 --cpu-baseline-seconds 0 --no-f32-mode --pmc-pass --json-out $O/b1_${v}_$i.json > $O/b1_${v}_$i.log 2>&1 || { tail -5 $O/b1_${v}_$i.log; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b1_${v}_$i.json')); s=d['stages_ms_per_step']; print('b1 $v', d['value'], d['ms_per_step'], 'fc1', s.get('fc1'))"
  done
done
