#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ragged.py tests/test_gpu_parity.py -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -rf -x -q > gpurun_out/pytest_ragged.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_ragged.log
if [ $rc -ne 0 ]; then exit $rc; fi
for w in yodas2 mls; do
timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 2 --cpu-baseline-seconds 0 --no-f32-mode --json-out gpurun_out/bench_$w.json > gpurun_out/bench_$w.log 2>&1 || { echo $w failed; tail -5 gpurun_out/bench_$w.log; exit 5; }
python -c "import json;d=json.load(open('gpurun_out/bench_$w.json'));print('$w',d['value'],d['ms_per_step'],d['whole_encode']['device_ms_per_step'], {k:v for k,v in d['stages_ms_per_step'].items() if k in ('down_s0','down_s1','down_s2','qkv','fc1','rvq','attention')})"
done
ROUNDS=2 KEYS="down_s1 qkv fc1" bash tools/ab_lib.sh
