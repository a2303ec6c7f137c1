#!/bin/bash
# Stage-time A/B of diagnostic / candidate builds: LIBS="d1 d2 d3" (tools/bin/libmimi_hip_<x>.so; "cur" = in-tree).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for l in ${LIBS:-cur}; do
  if [ $l = cur ]; then unset MIMI_HIP_LIB; else export MIMI_HIP_LIB=$GRAFT_REPO_ROOT/tools/bin/libmimi_hip_$l.so; fi
  timeout -k 10 200 python bench.py --cpu-baseline-seconds 0 --no-f32-mode --steps 10 --warmup 3 ${BENCH_ARGS:-} > gpurun_out/diag_$l.json 2>gpurun_out/diag_$l.err || { echo "bench $l failed"; tail -5 gpurun_out/diag_$l.err; exit 5; }
  python -c "import json; d=json.loads(open('gpurun_out/diag_$l.json').read().strip().splitlines()[-1]); s=d.get('stages_ms_per_step',{}); print('$l', d['value'], d['ms_per_step'], {k: s[k] for k in sorted(s) if k.startswith(('${KEYS:-res_down}'))})"
done
unset MIMI_HIP_LIB
if [ -n "${TESTLIB:-}" ]; then
  MIMI_HIP_LIB=$GRAFT_REPO_ROOT/tools/bin/libmimi_hip_$TESTLIB.so timeout -k 10 300 python -u -m pytest tests/test_stage0_fused.py -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread -rf -x -q > gpurun_out/pytest_diag.log 2>&1; echo "pytest($TESTLIB) rc=$?"; tail -3 gpurun_out/pytest_diag.log
fi
