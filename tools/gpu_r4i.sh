#!/bin/bash
# round 4: batch-1 LayerNorm-prologue tile A/B for q/k/v (ln_fused 1 = LayerNorm launch, 2/3/4 = prologue 16x64/32x64/16x128)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_ln_fused.py > gpurun_out/r4i_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r4i_pytest.log; exit 1; }
tail -1 gpurun_out/r4i_pytest.log
for L in 1 2 3 4 1 3 4; do
  timeout -k 10 200 python -u bench.py --batch 1 --steps 40 --cpu-baseline-seconds 0 --no-f32-mode --ln-fused $L --json-out gpurun_out/r4i_b1_ln$L.json > gpurun_out/r4i_b1_ln$L.log 2>&1 || { echo "bench ln$L failed"; tail -30 gpurun_out/r4i_b1_ln$L.log; exit 2; }
  python - $L <<'P'
import json,sys; l=sys.argv[1]; d=json.load(open(f"gpurun_out/r4i_b1_ln{l}.json")); s=d["stages_ms_per_step"]
print("ln_fused", l, d["value"], d["ms_per_step"], {k: s.get(k) for k in ("layernorm","qkv","fc1")})
P
done
