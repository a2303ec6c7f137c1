#!/bin/bash
# Round-5 session Z: v_pk_fma_f32 under concurrent load.  Three builds of the same sources: pk (the Makefile's flags
# at HEAD), noslp (ops.hip without SLP vectorisation: no packed FMAs in ops.hip), nopk (every object built without
# packed f32 ops).  tools/race_taps.py per build (engine A's taps vs A alone while a clone loads the GPU), codes
# bitwise across builds, then B = 32 and batch 1 timing alternated.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r5z"
mkdir -p "$O"
cd "$R"
for v in pk noslp nopk pk noslp nopk; do
  MIMI_HIP_LIB=$R/ab/libmimi_hip_$v.so timeout -k 10 200 python -u tools/race_taps.py 300 nocontrols > $O/taps_$v.log 2>&1 || { tail -5 $O/taps_$v.log; exit 1; }
  echo "taps $v: $(grep -c '^loaded' $O/taps_$v.log) of 300 loaded reps differ, $(grep -c '^idle' $O/taps_$v.log) idle"
done
for v in pk noslp nopk; do
  MIMI_HIP_LIB=$R/ab/libmimi_hip_$v.so timeout -k 10 200 python3 tools/lib_codes.py r5z_$v > $O/codes_$v.log 2>&1 || { tail -5 $O/codes_$v.log; exit 1; }
done
python3 tools/cmp_codes.py r5z_pk r5z_noslp && python3 tools/cmp_codes.py r5z_pk r5z_nopk || exit 1
for i in 1 2; do
  for v in pk noslp nopk; do
    export MIMI_HIP_LIB=$R/ab/libmimi_hip_$v.so
    timeout -k 10 200 python -u bench.py --steps 20 --cpu-baseline-seconds 0 --no-f32-mode --json-out $O/b32_${v}_$i.json > $O/b32_${v}_$i.log 2>&1 || { tail -5 $O/b32_${v}_$i.log; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b32_${v}_$i.json')); print('b32 $v', d['value'], d['ms_per_step'])"
    timeout -k 10 200 python -u bench.py --batch 1 --steps 30 --cpu-baseline-seconds 0 --no-f32-mode --json-out $O/b1_${v}_$i.json > $O/b1_${v}_$i.log 2>&1 || { tail -5 $O/b1_${v}_$i.log; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b1_${v}_$i.json')); print('b1 $v', d['value'], d['ms_per_step'])"
  done
done
unset MIMI_HIP_LIB
python3 - <<'PY'
import json, glob
def st(f): return json.load(open(f))['stages_ms_per_step']
for tag in ("b32", "b1"):
    runs = {v: [st(f) for f in sorted(glob.glob(f"gpurun_out/r5z/{tag}_{v}_*.json"))] for v in ("pk", "noslp", "nopk")}
    for k in runs["pk"][0]:
        m = {v: sum(x[k] for x in r) / len(r) for v, r in runs.items()}
        print(f"{tag} {k:14s} pk {m['pk']:.3f} noslp {m['noslp']:.3f} nopk {m['nopk']:.3f}")
PY
