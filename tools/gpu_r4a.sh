#!/bin/bash
# round-4 first check: the changed GPU tests, then the bench with the drop-in rate lines
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_ragged.py \
  "tests/test_gpu_parity.py::test_precision_modes" > gpurun_out/r4a_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r4a_pytest.log; exit 1; }
tail -3 gpurun_out/r4a_pytest.log
timeout -k 10 400 python -u bench.py --cpu-baseline-seconds 4 --json-out gpurun_out/r4a_bench.json > gpurun_out/r4a_bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r4a_bench.log; exit 2; }
python - <<'P'
import json; d=json.load(open("gpurun_out/r4a_bench.json"))
print(d["value"], d["ms_per_step"], {k: d[k] for k in ("k32","b1_k8","per_utterance_k32","configs2_b64") if k in d})
P
