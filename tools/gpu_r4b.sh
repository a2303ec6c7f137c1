#!/bin/bash
# round 4: RVQ forms -- quantizer parity per form, then the bench A/B (K = 8 headline, K = 32, batch 1) per form
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  "tests/test_gpu_parity.py::test_quantizer_forms_bit_exact" "tests/test_gpu_parity.py::test_quantizer_bit_exact_on_reference_embedding" "tests/test_gpu_parity.py::test_kernel_options_identical_codes" \
  > gpurun_out/r4b_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r4b_pytest.log; exit 1; }
tail -3 gpurun_out/r4b_pytest.log
for F in 1 2 3 "2 --option sc1_out=7" "2 --option sc1_out=1" "2 --option sc1_out=2"; do
  timeout -k 10 300 python -u bench.py --cpu-baseline-seconds 0 --no-f32-mode --option rvq_form=$F --json-out "gpurun_out/r4b_bench_f${F// /_}.json" > "gpurun_out/r4b_bench_f${F// /_}.log" 2>&1 || { echo "bench f$F failed"; tail -30 "gpurun_out/r4b_bench_f${F// /_}.log"; exit 2; }
  python - "${F// /_}" <<'P'
import json,sys; f=sys.argv[1]; d=json.load(open(f"gpurun_out/r4b_bench_f{f}.json"))
sm=d["stages_ms_per_step"]; print("form", f, d["value"], d["ms_per_step"], {k: sm.get(k) for k in ("rvq","qkv","fc1","o_proj","fc2","attention")}, {k: d[k].get("value") for k in ("k32","b1_k8","per_utterance_k32","configs2_b64") if k in d})
P
done
