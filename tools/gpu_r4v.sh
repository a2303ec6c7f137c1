#!/bin/bash
# round 4: o_proj + residual + post-attention LayerNorm in one kernel (oproj_ln.hip) -- parity, then A/B
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_oproj_ln.py \
  "tests/test_gpu_parity.py::test_kernel_options_identical_codes" > gpurun_out/r4v_pytest.log 2>&1 || { echo "pytest failed"; grep -E "Error|assert" gpurun_out/r4v_pytest.log | head; tail -5 gpurun_out/r4v_pytest.log; exit 1; }
tail -2 gpurun_out/r4v_pytest.log
run() {  # tag, bench args...
  local tag=$1; shift
  timeout -k 10 300 python -u bench.py "$@" --cpu-baseline-seconds 0 --no-f32-mode --pmc-pass --json-out gpurun_out/r4v_$tag.json > gpurun_out/r4v_$tag.log 2>&1 || { echo "bench $tag failed"; tail -30 gpurun_out/r4v_$tag.log; exit 2; }
  python - $tag <<'P'
import json,sys; t=sys.argv[1]; d=json.load(open(f"gpurun_out/r4v_{t}.json"))
st=d["stages_ms_per_step"]
print(t, d["value"], d["ms_per_step"], {k: st.get(k) for k in ("layernorm","o_proj","o_proj_ln","qkv_attention","fc1")})
P
}
run o0 --option oproj_ln=0
run o1 --option oproj_ln=1
run o0b --option oproj_ln=0
run o1b --option oproj_ln=1
