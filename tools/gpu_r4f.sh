#!/bin/bash
# round 4: RVQ helpers (fast norms, staged exact re-score, prefetched scalars): parity, chain stamps, A/B
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  "tests/test_gpu_parity.py::test_quantizer_chain_small_grids" "tests/test_gpu_parity.py::test_kernel_options_identical_codes" \
  "tests/test_gpu_parity.py::test_quantizer_forms_bit_exact" "tests/test_gpu_parity.py::test_quantizer_bit_exact_on_reference_embedding" \
  > gpurun_out/r4f_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r4f_pytest.log; exit 1; }
tail -2 gpurun_out/r4f_pytest.log
MIMI_HIP_LIB=$GRAFT_REPO_ROOT/tools/bin/libmimi_hip_stamp.so timeout -k 10 120 python tools/rvq_stamp.py || exit 4
for C in 0 1; do
  timeout -k 10 200 python -u bench.py --batch 1 --num-quantizers 32 --steps 20 --cpu-baseline-seconds 0 --no-f32-mode --option rvq_chain=$C --json-out gpurun_out/r4f_b1k32_c$C.json > gpurun_out/r4f_b1k32_c$C.log 2>&1 || { echo "bench c$C failed"; tail -30 gpurun_out/r4f_b1k32_c$C.log; exit 2; }
  python - $C <<'P'
import json,sys; c=sys.argv[1]; e=json.load(open(f"gpurun_out/r4f_b1k32_c{c}.json"))
print("chain", c, "b1k32", e["value"], e["ms_per_step"], "rvq", e["stages_ms_per_step"].get("rvq"))
P
done
timeout -k 10 300 python -u bench.py --cpu-baseline-seconds 0 --no-f32-mode --json-out gpurun_out/r4f_b32.json > gpurun_out/r4f_b32.log 2>&1 || { echo "bench b32 failed"; tail -30 gpurun_out/r4f_b32.log; exit 3; }
python - <<'P'
import json; d=json.load(open("gpurun_out/r4f_b32.json"))
print("b32", d["value"], d["ms_per_step"], "rvq", d["stages_ms_per_step"].get("rvq"), {k: d[k].get("value") for k in ("k32","b1_k8","per_utterance_k32","configs2_b64")})
P
