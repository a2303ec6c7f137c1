#!/bin/bash
# round 4: LayerNorm rows per wave A/B (B = 32 headline)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for R in 2 4 8 1 2 4; do
  timeout -k 10 300 python -u bench.py --cpu-baseline-seconds 0 --no-f32-mode --pmc-pass --option ln_rpw=$R --json-out gpurun_out/r4h_ln$R.json > gpurun_out/r4h_ln$R.log 2>&1 || { echo "bench ln$R failed"; tail -30 gpurun_out/r4h_ln$R.log; exit 2; }
  python - $R <<'P'
import json,sys; r=sys.argv[1]; d=json.load(open(f"gpurun_out/r4h_ln{r}.json"))
print("ln_rpw", r, d["value"], d["ms_per_step"], "layernorm", d["stages_ms_per_step"].get("layernorm"))
P
done
