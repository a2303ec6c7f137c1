#!/bin/bash
# round 4: residual epilogues with R loaded before the K loop (gemm_planes.h RPF): parity at HEAD (full GPU suite), A/B
# against the build without it (tools/bin/libmimi_hip_rpf0.so) at B = 32 and B = 1
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r4ab_pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|assert" gpurun_out/r4ab_pytest_gpu.log | head; tail -5 gpurun_out/r4ab_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r4ab_pytest_gpu.log
run() {  # tag, lib, bench args...
  local tag=$1 lib=$2; shift 2
  timeout -k 10 300 env MIMI_HIP_LIB=$PWD/tools/bin/$lib python -u bench.py "$@" --cpu-baseline-seconds 0 --no-f32-mode --pmc-pass --json-out gpurun_out/r4ab_$tag.json > gpurun_out/r4ab_$tag.log 2>&1 || { echo "bench $tag failed"; tail -30 gpurun_out/r4ab_$tag.log; exit 2; }
  python - $tag <<'P'
import json,sys; t=sys.argv[1]; d=json.load(open(f"gpurun_out/r4ab_{t}.json"))
st=d["stages_ms_per_step"]
print(t, d["value"], d["ms_per_step"], {k: st.get(k) for k in ("res1_s2","res1_s3","o_proj","fc2","res_s1")})
P
}
run r0 libmimi_hip_rpf0.so
run r1 libmimi_hip_rpf1.so
run r0b libmimi_hip_rpf0.so
run r1b libmimi_hip_rpf1.so
run b1r0 libmimi_hip_rpf0.so --batch 1 --steps 40
run b1r1 libmimi_hip_rpf1.so --batch 1 --steps 40
