#!/bin/bash
# Round-5 session AK: resblock.hip built without SLP vectorisation (ab/libmimi_hip_rsns.so) vs HEAD: codes bitwise,
# then B = 32 and batch 1 alternated with stage times
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r5ak"
mkdir -p "$O"
cd "$R"
MIMI_HIP_LIB=$R/ab/libmimi_hip_head.so timeout -k 10 200 python3 tools/lib_codes.py r5ak_head > $O/codes_head.log 2>&1 || { tail -5 $O/codes_head.log; exit 1; }
MIMI_HIP_LIB=$R/ab/libmimi_hip_rsns.so timeout -k 10 200 python3 tools/lib_codes.py r5ak_rsns > $O/codes_rsns.log 2>&1 || { tail -5 $O/codes_rsns.log; exit 1; }
python3 tools/cmp_codes.py r5ak_head r5ak_rsns || exit 1
for i in 1 2; do
  for v in rsns head; do
    export MIMI_HIP_LIB=$R/ab/libmimi_hip_$v.so
    timeout -k 10 200 python -u bench.py --steps 20 --cpu-baseline-seconds 0 --no-f32-mode --json-out $O/b32_${v}_$i.json > $O/b32_${v}_$i.log 2>&1 || { tail -5 $O/b32_${v}_$i.log; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b32_${v}_$i.json')); s=d['stages_ms_per_step']; print('b32 $v', d['value'], d['ms_per_step'], 'res_s1', s['res_s1'], 'res3_s2', s['res3_s2'])"
    timeout -k 10 200 python -u bench.py --batch 1 --steps 40 --cpu-baseline-seconds 0 --no-f32-mode --json-out $O/b1_${v}_$i.json > $O/b1_${v}_$i.log 2>&1 || { tail -5 $O/b1_${v}_$i.log; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b1_${v}_$i.json')); s=d['stages_ms_per_step']; print('b1 $v', d['value'], d['ms_per_step'], 'res_s1', s['res_s1'])"
  done
done
