#!/bin/bash
# Round-5 session W: every kernel compiled with -mllvm -amdgpu-sched-strategy=max-ilp (ab/libmimi_hip_ilp.so) vs the
# default scheduler (HEAD): codes bitwise, then B = 32 (stage times) and batch-1 alternated
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r5w"
mkdir -p "$O"
cd "$R"
timeout -k 10 200 python3 tools/lib_codes.py r5w_def > $O/codes_def.log 2>&1 || { tail -5 $O/codes_def.log; exit 1; }
MIMI_HIP_LIB=$R/ab/libmimi_hip_ilp.so timeout -k 10 200 python3 tools/lib_codes.py r5w_ilp > $O/codes_ilp.log 2>&1 || { tail -5 $O/codes_ilp.log; exit 1; }
python3 tools/cmp_codes.py r5w_def r5w_ilp || exit 1
for i in 1 2; do
  for v in ilp def; do
    if [ $v = ilp ]; then export MIMI_HIP_LIB=$R/ab/libmimi_hip_ilp.so; else unset MIMI_HIP_LIB; fi
    timeout -k 10 200 python -u bench.py --steps 20 --cpu-baseline-seconds 0 --no-f32-mode --pmc-pass --json-out $O/b32_${v}_$i.json > $O/b32_${v}_$i.log 2>&1 || { tail -5 $O/b32_${v}_$i.log; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b32_${v}_$i.json')); print('b32 $v', d['value'], d['ms_per_step'])"
    timeout -k 10 200 python -u bench.py --batch 1 --steps 30 --cpu-baseline-seconds 0 --no-f32-mode --pmc-pass --json-out $O/b1_${v}_$i.json > $O/b1_${v}_$i.log 2>&1 || { tail -5 $O/b1_${v}_$i.log; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b1_${v}_$i.json')); print('b1 $v', d['value'], d['ms_per_step'])"
  done
done
python3 - <<'PY'
import json, glob
def st(f): return json.load(open(f))['stages_ms_per_step']
for tag in ("b32", "b1"):
    a = [st(f) for f in sorted(glob.glob(f"gpurun_out/r5w/{tag}_def_*.json"))]
    b = [st(f) for f in sorted(glob.glob(f"gpurun_out/r5w/{tag}_ilp_*.json"))]
    for k in a[0]:
        da = sum(x[k] for x in a) / len(a); db = sum(x[k] for x in b) / len(b)
        print(f"{tag} {k:14s} def {da:.3f} ilp {db:.3f} {db - da:+.3f}")
PY
