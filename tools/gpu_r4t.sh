#!/bin/bash
# round 4: fused q/k/v + attention forming its input LayerNorm (qkv_attn_ln) -- parity, A/B
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_qkv_attn.py \
  "tests/test_gpu_parity.py::test_kernel_options_identical_codes" > gpurun_out/r4t_pytest.log 2>&1 || { echo "pytest failed"; grep -E "Error|assert" gpurun_out/r4t_pytest.log | head; tail -5 gpurun_out/r4t_pytest.log; exit 1; }
tail -2 gpurun_out/r4t_pytest.log
run() {  # tag, bench args...
  local tag=$1; shift
  timeout -k 10 300 python -u bench.py "$@" --cpu-baseline-seconds 0 --no-f32-mode --pmc-pass --json-out gpurun_out/r4t_$tag.json > gpurun_out/r4t_$tag.log 2>&1 || { echo "bench $tag failed"; tail -30 gpurun_out/r4t_$tag.log; exit 2; }
  python - $tag <<'P'
import json,sys; t=sys.argv[1]; d=json.load(open(f"gpurun_out/r4t_{t}.json"))
st=d["stages_ms_per_step"]
print(t, d["value"], d["ms_per_step"], {k: st.get(k) for k in ("layernorm","qkv_attention")})
P
}
run ln0 --option qkv_attn_ln=0
run ln1 --option qkv_attn_ln=1
run ln0b --option qkv_attn_ln=0
run ln1b --option qkv_attn_ln=1
