#!/bin/bash
# round 4: sc1 output stores on the conv GEMMs (MIMI_SC1_CONV 1 k1 convs, 2 k3 convs, 4 down convs) vs HEAD: same bits
# (codes of fixed batches from each build), A/B
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L0=$PWD/tokenize-audio_amd/mimi_hip/libmimi_hip.so
timeout -k 10 300 env MIMI_HIP_LIB=$L0 python -u tools/lib_codes.py s0 > gpurun_out/r4ag_codes.log 2>&1 || { echo "codes s0 failed"; tail -20 gpurun_out/r4ag_codes.log; exit 1; }
for V in 1 2 4; do
  timeout -k 10 300 env MIMI_HIP_LIB=$PWD/tools/bin/libmimi_hip_sc$V.so python -u tools/lib_codes.py s$V >> gpurun_out/r4ag_codes.log 2>&1 || { echo "codes s$V failed"; tail -20 gpurun_out/r4ag_codes.log; exit 1; }
done
python tools/cmp_codes.py s0 s1 s2 s4 || exit 3
run() {  # tag, lib
  local tag=$1 lib=$2; shift 2
  timeout -k 10 300 env MIMI_HIP_LIB=$lib python -u bench.py --cpu-baseline-seconds 0 --no-f32-mode --pmc-pass --json-out gpurun_out/r4ag_$tag.json > gpurun_out/r4ag_$tag.log 2>&1 || { echo "bench $tag failed"; tail -30 gpurun_out/r4ag_$tag.log; exit 2; }
  python - $tag <<'P'
import json,sys; t=sys.argv[1]; d=json.load(open(f"gpurun_out/r4ag_{t}.json"))
st=d["stages_ms_per_step"]
print(t, d["value"], d["ms_per_step"], {k: st.get(k) for k in ("res1_s2","res1_s3","res3_s2","res3_s3","down_s1","down_s2","down_s3")})
P
}
run s0 $L0
for V in 1 2 4; do run s$V $PWD/tools/bin/libmimi_hip_sc$V.so; done
run s0b $L0
for V in 1 2 4; do run s${V}b $PWD/tools/bin/libmimi_hip_sc$V.so; done
