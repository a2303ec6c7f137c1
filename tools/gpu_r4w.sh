#!/bin/bash
# round 4: fused q/k/v + attention retiring 2 W stages per barrier (QA_KG = 2, default) vs 1 (tools/bin/libmimi_hip_kg1.so)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_qkv_attn.py > gpurun_out/r4w_pytest.log 2>&1 || { echo "pytest failed"; grep -E "Error|assert" gpurun_out/r4w_pytest.log | head; tail -5 gpurun_out/r4w_pytest.log; exit 1; }
tail -2 gpurun_out/r4w_pytest.log
run() {  # tag, env assignment
  local tag=$1 ev=$2; shift 2
  timeout -k 10 300 env "$ev" python -u bench.py "$@" --cpu-baseline-seconds 0 --no-f32-mode --pmc-pass --json-out gpurun_out/r4w_$tag.json > gpurun_out/r4w_$tag.log 2>&1 || { echo "bench $tag failed"; tail -30 gpurun_out/r4w_$tag.log; exit 2; }
  python - $tag <<'P'
import json,sys; t=sys.argv[1]; d=json.load(open(f"gpurun_out/r4w_{t}.json"))
st=d["stages_ms_per_step"]
print(t, d["value"], d["ms_per_step"], {k: st.get(k) for k in ("qkv_attention",)})
P
}
run kg2 MIMI_HIP_LIB=$PWD/tokenize-audio_amd/mimi_hip/libmimi_hip.so
run kg1 MIMI_HIP_LIB=$PWD/tools/bin/libmimi_hip_kg1.so
run kg2b MIMI_HIP_LIB=$PWD/tokenize-audio_amd/mimi_hip/libmimi_hip.so
run kg1b MIMI_HIP_LIB=$PWD/tools/bin/libmimi_hip_kg1.so
