#!/bin/bash
# round 4: fused q/k/v + attention, attention-phase timing (QA_DIAG 1 / 8 / 16 / 24 builds)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() {  # tag, env assignment
  local tag=$1 ev=$2; shift 2
  timeout -k 10 300 env "$ev" python -u bench.py "$@" --cpu-baseline-seconds 0 --no-f32-mode --pmc-pass --json-out gpurun_out/r4u_$tag.json > gpurun_out/r4u_$tag.log 2>&1 || { echo "bench $tag failed"; tail -30 gpurun_out/r4u_$tag.log; exit 2; }
  python - $tag <<'P'
import json,sys; t=sys.argv[1]; d=json.load(open(f"gpurun_out/r4u_{t}.json"))
st=d["stages_ms_per_step"]
print(t, d["ms_per_step"], {k: st.get(k) for k in ("qkv_attention",)})
P
}
run full MIMI_HIP_LIB=$PWD/tokenize-audio_amd/mimi_hip/libmimi_hip.so
run d1 MIMI_HIP_LIB=$PWD/tools/bin/libmimi_hip_qa1.so
run d8 MIMI_HIP_LIB=$PWD/tools/bin/libmimi_hip_qa8.so
run d16 MIMI_HIP_LIB=$PWD/tools/bin/libmimi_hip_qa16.so
run d24 MIMI_HIP_LIB=$PWD/tools/bin/libmimi_hip_qa24.so
