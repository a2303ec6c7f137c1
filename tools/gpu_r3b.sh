#!/bin/bash
# ragged tests first (new code: fail fast), then the whole GPU suite, smoke, benches of the three workloads
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ragged.py -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf -x > gpurun_out/pytest_ragged.log 2>&1
rc=$?; echo "ragged pytest rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_ragged.log | tail -12
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -8
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -5 gpurun_out/smoke.log; exit 3; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_b32.json > gpurun_out/bench.log 2>&1 || { echo bench failed; tail -5 gpurun_out/bench.log; exit 4; }
python -c "import json;d=json.load(open('gpurun_out/bench_b32.json'));print('b32',d['value'],d.get('configs2_b64',{}).get('value'),d['roofline']['frac'])"
timeout -k 10 300 python bench.py --workload yodas2 --steps 10 --warmup 2 --cpu-baseline-seconds 0 --no-f32-mode --json-out gpurun_out/bench_yodas2.json > gpurun_out/bench_yodas2.log 2>&1 || { echo yodas2 failed; tail -5 gpurun_out/bench_yodas2.log; exit 5; }
python -c "import json;d=json.load(open('gpurun_out/bench_yodas2.json'));print('yodas2',d['value'],d['ms_per_step'])"
timeout -k 10 300 python bench.py --workload mls --steps 10 --warmup 2 --cpu-baseline-seconds 0 --no-f32-mode --json-out gpurun_out/bench_mls.json > gpurun_out/bench_mls.log 2>&1 || { echo mls failed; tail -5 gpurun_out/bench_mls.log; exit 6; }
python -c "import json;d=json.load(open('gpurun_out/bench_mls.json'));print('mls',d['value'],d['ms_per_step'])"
