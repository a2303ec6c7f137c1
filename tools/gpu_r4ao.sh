#!/bin/bash
# round 4: o_proj (and, in v3, fc2) on 64x128 tiles with loader waves (504 workgroups, two per CU) vs HEAD's 128x128:
# same bits (codes of fixed batches), A/B at B = 32
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L0=$PWD/tokenize-audio_amd/mimi_hip/libmimi_hip.so
timeout -k 10 300 env MIMI_HIP_LIB=$L0 python -u tools/lib_codes.py o0 > gpurun_out/r4ao_codes.log 2>&1 || { echo "codes o0 failed"; tail -20 gpurun_out/r4ao_codes.log; exit 1; }
for V in 1 2 3; do
  timeout -k 10 300 env MIMI_HIP_LIB=$PWD/tools/bin/libmimi_hip_op$V.so python -u tools/lib_codes.py o$V >> gpurun_out/r4ao_codes.log 2>&1 || { echo "codes o$V failed"; tail -20 gpurun_out/r4ao_codes.log; exit 1; }
done
python tools/cmp_codes.py o0 o1 o2 o3 || exit 3
run() {  # tag, lib
  local tag=$1 lib=$2; shift 2
  timeout -k 10 300 env MIMI_HIP_LIB=$lib python -u bench.py --cpu-baseline-seconds 0 --no-f32-mode --pmc-pass --json-out gpurun_out/r4ao_$tag.json > gpurun_out/r4ao_$tag.log 2>&1 || { echo "bench $tag failed"; tail -30 gpurun_out/r4ao_$tag.log; exit 2; }
  python - $tag <<'P' || true
import json,sys; t=sys.argv[1]; d=json.load(open(f"gpurun_out/r4ao_{t}.json"))
st=d["stages_ms_per_step"]
print(t, d["value"], d["ms_per_step"], {k: st.get(k) for k in ("o_proj","fc2")})
P
}
for r in a b; do
  run o0$r $L0
  for V in 1 2 3; do run o$V$r $PWD/tools/bin/libmimi_hip_op$V.so; done
done
