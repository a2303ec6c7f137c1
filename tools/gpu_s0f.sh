#!/bin/bash
# Fused stage-0 check: bitwise tests of the 3 variants, then bench A/B of the variants (B = 32 x 10 s).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_stage0_fused.py -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread -rf -x -v > gpurun_out/pytest_s0f.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -12 gpurun_out/pytest_s0f.log
if [ $rc -ne 0 ]; then exit $rc; fi
for r in 1 2; do
for v in 0 1; do
timeout -k 10 200 python bench.py --cpu-baseline-seconds 0 --no-f32-mode --steps 20 --warmup 5 --stage0-fused $v > gpurun_out/s0f_$v.json 2>gpurun_out/s0f_$v.err || { echo "bench $v failed"; tail -5 gpurun_out/s0f_$v.err; exit 5; }
python -c "import json; d=json.loads(open('gpurun_out/s0f_$v.json').read().strip().splitlines()[-1]); s=d.get('stages_ms_per_step',{}); print('v$v', d['value'], d['ms_per_step'], {k: s[k] for k in sorted(s) if k.startswith(('down_s0','res_s0','res_down','res_s1'))})"
done
done
