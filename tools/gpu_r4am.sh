#!/bin/bash
# round 4 check at HEAD (quantizer small tiles): full GPU suite, smoke, one default bench line
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r4am_pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|assert" gpurun_out/r4am_pytest_gpu.log | head; tail -5 gpurun_out/r4am_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r4am_pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4am_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r4am_smoke.log; exit 2; }
tail -1 gpurun_out/r4am_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r4am_bench.json 2> gpurun_out/r4am_bench.err || { echo "bench failed"; tail -20 gpurun_out/r4am_bench.err; exit 3; }
python - <<'P'
import json; d=json.loads(open("gpurun_out/r4am_bench.json").read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d["k32"], d["b1_k8"], d["configs2_b64"], d["cpu_baseline"]["value"])
P
