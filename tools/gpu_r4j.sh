#!/bin/bash
# round 4: RVQ XCD grouping -- parity, A/B, and the FETCH/WRITE passes at HEAD
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  "tests/test_gpu_parity.py::test_kernel_options_identical_codes" "tests/test_gpu_parity.py::test_quantizer_forms_bit_exact" \
  "tests/test_gpu_parity.py::test_full_size_batch_properties" > gpurun_out/r4j_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r4j_pytest.log; exit 1; }
tail -1 gpurun_out/r4j_pytest.log
for X in 0 1 0 1; do
  timeout -k 10 300 python -u bench.py --cpu-baseline-seconds 0 --no-f32-mode --option rvq_xcd=$X --json-out gpurun_out/r4j_x$X.json > gpurun_out/r4j_x$X.log 2>&1 || { echo "bench x$X failed"; tail -30 gpurun_out/r4j_x$X.log; exit 2; }
  python - $X <<'P'
import json,sys; x=sys.argv[1]; d=json.load(open(f"gpurun_out/r4j_x{x}.json"))
print("rvq_xcd", x, d["value"], d["ms_per_step"], "rvq", d["stages_ms_per_step"].get("rvq"), "k32", d["k32"]["value"])
P
done
TAG=r4b STEPS=10 bash tools/profile_round.sh || exit 3
