#!/bin/bash
# Round-5 session O: down convs (pair GEMM, large grids) as 4 compute waves of 128 x 64 (MIMI_DOWN_VARIANT=1) vs 8 of
# 64 x 64 (0): codes bitwise, then B = 32 bench alternated
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r5o"
mkdir -p "$O"
cd "$R"
for v in 0 1 2; do
  MIMI_DOWN_VARIANT=$v timeout -k 10 200 python3 tools/lib_codes.py r5o_dv$v > $O/codes_$v.log 2>&1 || { tail -5 $O/codes_$v.log; exit 1; }
done
python3 tools/cmp_codes.py r5o_dv0 r5o_dv1 r5o_dv2 || exit 1
for i in 1 2; do
  for v in 0 1 2; do
    MIMI_DOWN_VARIANT=$v timeout -k 10 200 python -u bench.py --steps 20 --cpu-baseline-seconds 0 --no-f32-mode --pmc-pass --json-out $O/b32_${v}_$i.json > $O/b32_${v}_$i.log 2>&1 || { tail -5 $O/b32_${v}_$i.log; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b32_${v}_$i.json')); s=d['stages_ms_per_step']; print('dv $v', d['value'], d['ms_per_step'], {k: s[k] for k in ('down_s1','down_s2','down_s3')})"
  done
done
