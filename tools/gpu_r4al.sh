#!/bin/bash
# round 4: small-grid tiles below one 128x128 workgroup per CU for more roles (MIMI_SMALL_ROLES: 1 downsample +
# input_proj (HEAD), 2 o_proj, 4 fc2, 8 final conv): same bits (codes of fixed batches), A/B at B = 32
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for V in 1 3 5 9; do
  timeout -k 10 300 env MIMI_HIP_LIB=$PWD/tools/bin/libmimi_hip_sr$V.so python -u tools/lib_codes.py r$V >> gpurun_out/r4al_codes.log 2>&1 || { echo "codes r$V failed"; tail -20 gpurun_out/r4al_codes.log; exit 1; }
done
python tools/cmp_codes.py r1 r3 r5 r9 || exit 3
run() {  # tag, lib
  local tag=$1 lib=$2; shift 2
  timeout -k 10 300 env MIMI_HIP_LIB=$lib python -u bench.py --cpu-baseline-seconds 0 --no-f32-mode --pmc-pass --json-out gpurun_out/r4al_$tag.json > gpurun_out/r4al_$tag.log 2>&1 || { echo "bench $tag failed"; tail -30 gpurun_out/r4al_$tag.log; exit 2; }
  python - $tag <<'P' || true
import json,sys; t=sys.argv[1]; d=json.load(open(f"gpurun_out/r4al_{t}.json"))
st=d["stages_ms_per_step"]
print(t, d["value"], d["ms_per_step"], {k: st.get(k) for k in ("downsample","input_proj","o_proj","fc2","final")})
P
}
for r in a b; do
  for V in 1 3 5 9; do run r$V$r $PWD/tools/bin/libmimi_hip_sr$V.so; done
done
