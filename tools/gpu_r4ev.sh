#!/bin/bash
# round-4 evidence at HEAD: rocprofv3 trace + stats + FETCH/WRITE PMC (profile_round.sh), SQ/GRBM passes, then the
# bench lines (B = 32 with the CPU baseline, B = 1, B = 4, yodas2, mls) and smoke
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${TAG:-r4a}
TAG=$T STEPS=10 bash tools/profile_round.sh || exit 1
PASSES="SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,GRBM_GUI_ACTIVE;SQ_WAVE_CYCLES,SQ_WAIT_INST_LDS,SQ_VALU_MFMA_BUSY_CYCLES,SQ_LDS_BANK_CONFLICT,GRBM_GUI_ACTIVE" TAG=pmc_sq_$T bash tools/pmc_pass.sh || exit 2
python tools/sq_table.py pmc_sq_$T > gpurun_out/${T}_sq_counters.txt || exit 3
timeout -k 10 400 python -u bench.py --json-out gpurun_out/${T}_bench_b32.json > gpurun_out/${T}_bench_b32.log 2>&1 || { echo "bench b32 failed"; tail -20 gpurun_out/${T}_bench_b32.log; exit 4; }
timeout -k 10 200 python -u bench.py --batch 1 --steps 40 --cpu-baseline-seconds 0 --no-f32-mode --json-out gpurun_out/${T}_bench_b1.json > gpurun_out/${T}_bench_b1.log 2>&1 || exit 5
timeout -k 10 200 python -u bench.py --batch 4 --steps 20 --cpu-baseline-seconds 0 --no-f32-mode --json-out gpurun_out/${T}_bench_b4.json > gpurun_out/${T}_bench_b4.log 2>&1 || exit 6
timeout -k 10 300 python -u bench.py --workload yodas2 --steps 10 --cpu-baseline-seconds 0 --json-out gpurun_out/${T}_bench_yodas2.json > gpurun_out/${T}_bench_yodas2.log 2>&1 || exit 7
timeout -k 10 300 python -u bench.py --workload mls --steps 10 --cpu-baseline-seconds 0 --json-out gpurun_out/${T}_bench_mls.json > gpurun_out/${T}_bench_mls.log 2>&1 || exit 8
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/${T}_smoke.log; exit 9; }
python - $T <<'P'
import json,sys; t=sys.argv[1]
for w in ("b32","b1","b4","yodas2","mls"):
    d=json.load(open(f"gpurun_out/{t}_bench_{w}.json"))
    x={k: (d[k].get("value") if isinstance(d.get(k),dict) else d.get(k)) for k in ("k32","b1_k8","per_utterance_k32","configs2_b64","f32_mode_value","pcie_inclusive_value")}
    print(w, d["value"], d["ms_per_step"], (d.get("roofline") or {}).get("frac"), x)
P
tail -1 gpurun_out/${T}_smoke.log
head -30 gpurun_out/${T}_sq_counters.txt
