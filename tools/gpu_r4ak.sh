#!/bin/bash
# round 4: downsample / input_proj on the small-grid tiles below one workgroup per CU (MIMI_DS_SMALL) vs HEAD: same
# bits (codes of fixed batches), A/B at B = 32 and B = 64
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L0=$PWD/tokenize-audio_amd/mimi_hip/libmimi_hip.so
L1=$PWD/tools/bin/libmimi_hip_ds1.so
timeout -k 10 300 env MIMI_HIP_LIB=$L0 python -u tools/lib_codes.py d0 > gpurun_out/r4ak_codes.log 2>&1 || { echo "codes d0 failed"; tail -20 gpurun_out/r4ak_codes.log; exit 1; }
timeout -k 10 300 env MIMI_HIP_LIB=$L1 python -u tools/lib_codes.py d1 >> gpurun_out/r4ak_codes.log 2>&1 || { echo "codes d1 failed"; tail -20 gpurun_out/r4ak_codes.log; exit 1; }
python tools/cmp_codes.py d0 d1 || exit 3
run() {  # tag, lib
  local tag=$1 lib=$2; shift 2
  timeout -k 10 300 env MIMI_HIP_LIB=$lib python -u bench.py --cpu-baseline-seconds 0 --no-f32-mode --pmc-pass --json-out gpurun_out/r4ak_$tag.json > gpurun_out/r4ak_$tag.log 2>&1 || { echo "bench $tag failed"; tail -30 gpurun_out/r4ak_$tag.log; exit 2; }
  python - $tag <<'P'
import json,sys; t=sys.argv[1]; d=json.load(open(f"gpurun_out/r4ak_{t}.json"))
st=d["stages_ms_per_step"]
print(t, d["value"], d["ms_per_step"], {k: st.get(k) for k in ("downsample","input_proj","rvq")}, "b64", d["configs2_b64"]["value"])
P
}
run d0 $L0
run d1 $L1
run d0b $L0
run d1b $L1
