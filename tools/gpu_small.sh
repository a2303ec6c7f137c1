#!/bin/bash
# small-batch check: GPU tests at the defaults, then bench A/B at B = 1 / 4 of the LayerNorm prologue (ln_fused) and
# the RVQ workgroup size on small grids (MIMI_RVQ_SMALL_WAVES)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${SMALL_TESTS:-tests} -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread -rf -x -v > gpurun_out/pytest_small.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAIL|ERROR" gpurun_out/pytest_small.log | tail -8
if [ $rc -ne 0 ]; then exit $rc; fi
for B in ${BATCHES:-1 4}; do
for r in 1 2; do
for cfg in ${CFGS:-"1 2" "0 8" "1 8" "1 4" "2 2"}; do
set -- $cfg
MIMI_RVQ_SMALL_WAVES=$2 timeout -k 10 200 python bench.py --batch $B --cpu-baseline-seconds 0 --no-f32-mode --steps 50 --warmup 10 --ln-fused $1 > gpurun_out/sm_${B}_$1_$2.json 2>gpurun_out/sm.err || { echo "bench $cfg failed"; tail -5 gpurun_out/sm.err; exit 5; }
python -c "import json; d=json.loads(open('gpurun_out/sm_${B}_$1_$2.json').read().strip().splitlines()[-1]); s=d.get('stages_ms_per_step',{}); print('B$B ln$1 rvqw$2', d['value'], d['ms_per_step'], {k: s[k] for k in sorted(s) if k in ('qkv','fc1','layernorm','rvq')})"
done
done
done
