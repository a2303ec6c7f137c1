#!/bin/bash
# LayerNorm-prologue check: bitwise tests (+ the ragged / parity suites), then bench A/B of ln_fused at B = 1 and 4
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest ${LNF_TESTS:-tests} -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread -rf -x -v > gpurun_out/pytest_lnf.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR" gpurun_out/pytest_lnf.log | tail -25
if [ $rc -ne 0 ]; then exit $rc; fi
for B in 1 4; do
for r in 1 2; do
for v in 0 1 2; do
timeout -k 10 200 python bench.py --batch $B --cpu-baseline-seconds 0 --no-f32-mode --steps 50 --warmup 10 --ln-fused $v > gpurun_out/lnf_${B}_$v.json 2>gpurun_out/lnf_$v.err || { echo "bench $v failed"; tail -5 gpurun_out/lnf_$v.err; exit 5; }
python -c "import json; d=json.loads(open('gpurun_out/lnf_${B}_$v.json').read().strip().splitlines()[-1]); s=d.get('stages_ms_per_step',{}); print('B$B v$v', d['value'], d['ms_per_step'], {k: s[k] for k in sorted(s) if k in ('qkv','fc1','layernorm','attention','rvq','fc2','o_proj')})"
done
done
done
