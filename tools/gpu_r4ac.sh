#!/bin/bash
# round 4: fused stage 0 with the block waves at raised issue priority (S0F_PRIO 1-3) vs none: parity + A/B
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 env MIMI_HIP_LIB=$PWD/tools/bin/libmimi_hip_s0p2.so python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_stage0_fused.py > gpurun_out/r4ac_pytest.log 2>&1 || { echo "pytest failed"; grep -E "Error|assert" gpurun_out/r4ac_pytest.log | head; tail -5 gpurun_out/r4ac_pytest.log; exit 1; }
tail -1 gpurun_out/r4ac_pytest.log
run() {  # tag, lib
  local tag=$1 lib=$2; shift 2
  timeout -k 10 300 env MIMI_HIP_LIB=$lib python -u bench.py --cpu-baseline-seconds 0 --no-f32-mode --pmc-pass --json-out gpurun_out/r4ac_$tag.json > gpurun_out/r4ac_$tag.log 2>&1 || { echo "bench $tag failed"; tail -30 gpurun_out/r4ac_$tag.log; exit 2; }
  python - $tag <<'P'
import json,sys; t=sys.argv[1]; d=json.load(open(f"gpurun_out/r4ac_{t}.json"))
st=d["stages_ms_per_step"]
print(t, d["value"], d["ms_per_step"], {k: st.get(k) for k in ("res_down_s0","res_s1")})
P
}
L0=$PWD/tokenize-audio_amd/mimi_hip/libmimi_hip.so
run p0 $L0
run p1 $PWD/tools/bin/libmimi_hip_s0p1.so
run p2 $PWD/tools/bin/libmimi_hip_s0p2.so
run p3 $PWD/tools/bin/libmimi_hip_s0p3.so
run p0b $L0
run p2b $PWD/tools/bin/libmimi_hip_s0p2.so
