#!/bin/bash
# round 4: fused q/k/v + attention -- bitwise parity vs the two-kernel path, then A/B of the B = 32 step
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_qkv_attn.py \
  > gpurun_out/r4k_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r4k_pytest.log; exit 1; }
tail -3 gpurun_out/r4k_pytest.log
for X in 0 1 0 1; do
  timeout -k 10 300 python -u bench.py --cpu-baseline-seconds 0 --no-f32-mode --option qkv_attn=$X --json-out gpurun_out/r4k_q$X.json > gpurun_out/r4k_q$X.log 2>&1 || { echo "bench q$X failed"; tail -30 gpurun_out/r4k_q$X.log; exit 2; }
  python - $X <<'P'
import json,sys; x=sys.argv[1]; d=json.load(open(f"gpurun_out/r4k_q{x}.json"))
st=d["stages_ms_per_step"]
print("qkv_attn", x, d["value"], d["ms_per_step"], {k: st.get(k) for k in ("qkv","attention","qkv_attention")}, "k32", d["k32"]["value"])
P
done
