#!/bin/bash
# round 4: fused q/k/v + attention with the W fragment reads software-pipelined (QA_SGB) and one opaque fragment base per
# step: parity (fused == two-kernel path, bitwise) and A/B against the previous build (tools/bin/libmimi_hip_qa_old.so)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for V in 2 3; do
  timeout -k 10 600 env MIMI_HIP_LIB=$PWD/tools/bin/libmimi_hip_sgb$V.so python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
    tests/test_qkv_attn.py > gpurun_out/r4z_pytest_sgb$V.log 2>&1 || { echo "pytest sgb$V failed"; grep -E "Error|assert" gpurun_out/r4z_pytest_sgb$V.log | head; tail -5 gpurun_out/r4z_pytest_sgb$V.log; exit 1; }
  tail -1 gpurun_out/r4z_pytest_sgb$V.log
done
run() {  # tag, lib
  local tag=$1 lib=$2
  timeout -k 10 300 env MIMI_HIP_LIB=$PWD/tools/bin/$lib python -u bench.py --cpu-baseline-seconds 0 --no-f32-mode --pmc-pass --json-out gpurun_out/r4z_$tag.json > gpurun_out/r4z_$tag.log 2>&1 || { echo "bench $tag failed"; tail -30 gpurun_out/r4z_$tag.log; exit 2; }
  python - $tag <<'P'
import json,sys; t=sys.argv[1]; d=json.load(open(f"gpurun_out/r4z_{t}.json"))
st=d["stages_ms_per_step"]
print(t, d["value"], d["ms_per_step"], {k: st.get(k) for k in ("qkv_attention","fc1","fc2","o_proj")})
P
}
run old libmimi_hip_qa_old.so
run sgb0 libmimi_hip_sgb0.so
run sgb2 libmimi_hip_sgb2.so
run sgb3 libmimi_hip_sgb3.so
run sgb4 libmimi_hip_sgb4.so
run oldb libmimi_hip_qa_old.so
run sgb2b libmimi_hip_sgb2.so
run sgb3b libmimi_hip_sgb3.so
