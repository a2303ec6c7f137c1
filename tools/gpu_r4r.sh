#!/bin/bash
# round 4: fused stage-2 block phase timing (RR_DIAG builds)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() {  # tag, env assignment, bench args...
  local tag=$1 ev=$2; shift 2
  timeout -k 10 300 env "$ev" python -u bench.py "$@" --cpu-baseline-seconds 0 --no-f32-mode --pmc-pass --json-out gpurun_out/r4r_$tag.json > gpurun_out/r4r_$tag.log 2>&1 || { echo "bench $tag failed"; tail -30 gpurun_out/r4r_$tag.log; exit 2; }
  python - $tag <<'P'
import json,sys; t=sys.argv[1]; d=json.load(open(f"gpurun_out/r4r_{t}.json"))
st=d["stages_ms_per_step"]
print(t, d["value"], d["ms_per_step"], {k: st.get(k) for k in ("down_s1","res_s2","res3_s2","res1_s2")})
P
}
run full MIMI_HIP_LIB=$PWD/tokenize-audio_amd/mimi_hip/libmimi_hip.so
run rr1 MIMI_HIP_LIB=$PWD/tools/bin/libmimi_hip_rr1.so
run rr2 MIMI_HIP_LIB=$PWD/tools/bin/libmimi_hip_rr2.so
run rr4 MIMI_HIP_LIB=$PWD/tools/bin/libmimi_hip_rr4.so
