#!/bin/bash
# round 4: RVQ forms 2/4/5/6 A/B (B = 32 K = 8 headline + k32 line; B = 1 K = 32 stage profile)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  "tests/test_gpu_parity.py::test_quantizer_forms_bit_exact" "tests/test_gpu_parity.py::test_kernel_options_identical_codes" \
  > gpurun_out/r4d_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r4d_pytest.log; exit 1; }
tail -2 gpurun_out/r4d_pytest.log
for F in 2 4 5 6; do
  timeout -k 10 300 python -u bench.py --cpu-baseline-seconds 0 --no-f32-mode --option rvq_form=$F --json-out gpurun_out/r4d_b32_f$F.json > gpurun_out/r4d_b32_f$F.log 2>&1 || { echo "bench f$F failed"; tail -30 gpurun_out/r4d_b32_f$F.log; exit 2; }
  timeout -k 10 200 python -u bench.py --batch 1 --num-quantizers 32 --steps 20 --cpu-baseline-seconds 0 --no-f32-mode --option rvq_form=$F --json-out gpurun_out/r4d_b1k32_f$F.json > gpurun_out/r4d_b1k32_f$F.log 2>&1 || { echo "bench b1 f$F failed"; tail -30 gpurun_out/r4d_b1k32_f$F.log; exit 3; }
  python - $F <<'P'
import json,sys; f=sys.argv[1]; d=json.load(open(f"gpurun_out/r4d_b32_f{f}.json")); e=json.load(open(f"gpurun_out/r4d_b1k32_f{f}.json"))
print("form", f, "b32", d["value"], d["stages_ms_per_step"].get("rvq"), "k32", d["k32"]["value"], "b1k8", d["b1_k8"]["value"], "utt", d["per_utterance_k32"]["value"], "| b1k32", e["value"], e["ms_per_step"], "rvq", e["stages_ms_per_step"].get("rvq"))
P
done
