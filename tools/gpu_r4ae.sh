#!/bin/bash
# round 4: down convs with planes output (down_s1 / s2) loading the next tile's first ring stages under the epilogue
# (FL_PF, tools/bin/libmimi_hip_dpf1.so) vs HEAD: parity + A/B
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 env MIMI_HIP_LIB=$PWD/tools/bin/libmimi_hip_dpf1.so python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/r4ae_pytest.log 2>&1 || { echo "pytest failed"; grep -E "Error|assert" gpurun_out/r4ae_pytest.log | head; tail -5 gpurun_out/r4ae_pytest.log; exit 1; }
tail -1 gpurun_out/r4ae_pytest.log
run() {  # tag, lib
  local tag=$1 lib=$2; shift 2
  timeout -k 10 300 env MIMI_HIP_LIB=$lib python -u bench.py --cpu-baseline-seconds 0 --no-f32-mode --pmc-pass --json-out gpurun_out/r4ae_$tag.json > gpurun_out/r4ae_$tag.log 2>&1 || { echo "bench $tag failed"; tail -30 gpurun_out/r4ae_$tag.log; exit 2; }
  python - $tag <<'P'
import json,sys; t=sys.argv[1]; d=json.load(open(f"gpurun_out/r4ae_{t}.json"))
st=d["stages_ms_per_step"]
print(t, d["value"], d["ms_per_step"], {k: st.get(k) for k in ("down_s1","down_s2","down_s3")})
P
}
L0=$PWD/tokenize-audio_amd/mimi_hip/libmimi_hip.so
run h0 $L0
run pf $PWD/tools/bin/libmimi_hip_dpf1.so
run h0b $L0
run pfb $PWD/tools/bin/libmimi_hip_dpf1.so
