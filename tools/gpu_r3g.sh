#!/bin/bash
# round-3 check at HEAD: whole GPU suite, smoke, the headline bench (B = 32; + B = 64 inside), B = 1, yodas2, mls
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -6
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -5 gpurun_out/smoke.log; exit 3; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_b32.json > gpurun_out/bench.log 2>&1 || { echo bench failed; tail -5 gpurun_out/bench.log; exit 4; }
python -c "import json;d=json.load(open('gpurun_out/bench_b32.json'));print('b32',d['value'],d['ms_per_step'],d.get('configs2_b64',{}).get('value'),d['roofline']['frac'],d['roofline']['traffic'])"
timeout -k 10 300 python bench.py --batch 1 --steps 50 --warmup 10 --cpu-baseline-seconds 0 --no-f32-mode --json-out gpurun_out/bench_b1.json > gpurun_out/bench_b1.log 2>&1 || { echo b1 failed; exit 5; }
python -c "import json;d=json.load(open('gpurun_out/bench_b1.json'));print('b1',d['value'],d['ms_per_step'])"
for w in yodas2 mls; do
timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 2 --cpu-baseline-seconds 0 --no-f32-mode --json-out gpurun_out/bench_$w.json > gpurun_out/bench_$w.log 2>&1 || { echo $w failed; tail -5 gpurun_out/bench_$w.log; exit 6; }
python -c "import json;d=json.load(open('gpurun_out/bench_$w.json'));print('$w',d['value'],d['ms_per_step'])"
done
