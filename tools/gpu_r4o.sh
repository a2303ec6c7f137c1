#!/bin/bash
# round 4: row-slab GEMMs (gemm_rows.h) -- bitwise parity vs the planes kernels, then A/B per role
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gemm_rows.py \
  "tests/test_gpu_parity.py::test_kernel_options_identical_codes" > gpurun_out/r4o_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r4o_pytest.log; exit 1; }
tail -2 gpurun_out/r4o_pytest.log
run() {  # tag, bench args...
  local tag=$1; shift
  timeout -k 10 300 python -u bench.py "$@" --cpu-baseline-seconds 0 --no-f32-mode --pmc-pass --json-out gpurun_out/r4o_$tag.json > gpurun_out/r4o_$tag.log 2>&1 || { echo "bench $tag failed"; tail -30 gpurun_out/r4o_$tag.log; exit 2; }
  python - $tag <<'P'
import json,sys; t=sys.argv[1]; d=json.load(open(f"gpurun_out/r4o_{t}.json"))
st=d["stages_ms_per_step"]
print(t, d["value"], d["ms_per_step"], {k: st.get(k) for k in ("fc1","fc2","o_proj","qkv_attention","layernorm")})
P
}
run r0 --option gemm_rows=0
run r7 --option gemm_rows=7
run r0b --option gemm_rows=0
run r7b --option gemm_rows=7
