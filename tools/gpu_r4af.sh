#!/bin/bash
# round 4: fc1 tile variants (MIMI_FC1_V 1-4: 128x128 / 256x128, persistent + next-tile prefetch, loader waves, sc1
# stores) vs HEAD's 128x128 2-stage tile: same bits (codes of fixed batches from each build), A/B
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L0=$PWD/tokenize-audio_amd/mimi_hip/libmimi_hip.so
timeout -k 10 300 env MIMI_HIP_LIB=$L0 python -u tools/lib_codes.py v0 > gpurun_out/r4af_codes.log 2>&1 || { echo "codes v0 failed"; tail -20 gpurun_out/r4af_codes.log; exit 1; }
for V in 1 2 3 4; do
  timeout -k 10 300 env MIMI_HIP_LIB=$PWD/tools/bin/libmimi_hip_fc1v$V.so python -u tools/lib_codes.py v$V >> gpurun_out/r4af_codes.log 2>&1 || { echo "codes v$V failed"; tail -20 gpurun_out/r4af_codes.log; exit 1; }
done
python tools/cmp_codes.py v0 v1 v2 v3 v4 || exit 3
run() {  # tag, lib
  local tag=$1 lib=$2; shift 2
  timeout -k 10 300 env MIMI_HIP_LIB=$lib python -u bench.py --cpu-baseline-seconds 0 --no-f32-mode --pmc-pass --json-out gpurun_out/r4af_$tag.json > gpurun_out/r4af_$tag.log 2>&1 || { echo "bench $tag failed"; tail -30 gpurun_out/r4af_$tag.log; exit 2; }
  python - $tag <<'P'
import json,sys; t=sys.argv[1]; d=json.load(open(f"gpurun_out/r4af_{t}.json"))
st=d["stages_ms_per_step"]
print(t, d["value"], d["ms_per_step"], {k: st.get(k) for k in ("fc1","fc2")})
P
}
run v0 $L0
for V in 1 2 3 4; do run v$V $PWD/tools/bin/libmimi_hip_fc1v$V.so; done
run v0b $L0
