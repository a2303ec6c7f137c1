#!/bin/bash
# round 4: persistent all-levels RVQ (rvq_chain) on small grids: parity, then batch-1 A/B
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  "tests/test_gpu_parity.py::test_quantizer_chain_small_grids" "tests/test_gpu_parity.py::test_kernel_options_identical_codes" \
  > gpurun_out/r4e_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r4e_pytest.log; exit 1; }
tail -2 gpurun_out/r4e_pytest.log
for C in 0 1; do
  timeout -k 10 200 python -u bench.py --batch 1 --num-quantizers 32 --steps 20 --cpu-baseline-seconds 0 --no-f32-mode --option rvq_chain=$C --json-out gpurun_out/r4e_b1k32_c$C.json > gpurun_out/r4e_b1k32_c$C.log 2>&1 || { echo "bench c$C failed"; tail -30 gpurun_out/r4e_b1k32_c$C.log; exit 2; }
  timeout -k 10 200 python -u bench.py --batch 1 --steps 20 --cpu-baseline-seconds 0 --no-f32-mode --option rvq_chain=$C --json-out gpurun_out/r4e_b1k8_c$C.json > gpurun_out/r4e_b1k8_c$C.log 2>&1 || { echo "bench k8 c$C failed"; tail -30 gpurun_out/r4e_b1k8_c$C.log; exit 3; }
  python - $C <<'P'
import json,sys; c=sys.argv[1]; e=json.load(open(f"gpurun_out/r4e_b1k32_c{c}.json")); d=json.load(open(f"gpurun_out/r4e_b1k8_c{c}.json"))
print("chain", c, "b1k32", e["value"], e["ms_per_step"], "rvq", e["stages_ms_per_step"].get("rvq"), "| b1k8", d["value"], d["ms_per_step"], "rvq", d["stages_ms_per_step"].get("rvq"))
P
done
