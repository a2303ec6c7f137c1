#!/bin/bash
# round 4: fc1 tile order in XCD column groups (engine option fc1_cg; gemm_planes.h GemmArgs::ncg): parity, A/B, fc1 fetch
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  "tests/test_gpu_parity.py::test_kernel_options_identical_codes" > gpurun_out/r4y_pytest.log 2>&1 || { echo "pytest failed"; grep -E "Error|assert" gpurun_out/r4y_pytest.log | head; tail -5 gpurun_out/r4y_pytest.log; exit 1; }
tail -2 gpurun_out/r4y_pytest.log
run() {  # tag, bench args...
  local tag=$1; shift
  timeout -k 10 300 python -u bench.py "$@" --cpu-baseline-seconds 0 --no-f32-mode --pmc-pass --json-out gpurun_out/r4y_$tag.json > gpurun_out/r4y_$tag.log 2>&1 || { echo "bench $tag failed"; tail -30 gpurun_out/r4y_$tag.log; exit 2; }
  python - $tag <<'P'
import json,sys; t=sys.argv[1]; d=json.load(open(f"gpurun_out/r4y_{t}.json"))
st=d["stages_ms_per_step"]
print(t, d["value"], d["ms_per_step"], {k: st.get(k) for k in ("fc1","fc2","o_proj","qkv_attention")})
P
}
run cg1 --option fc1_cg=1
run cg2 --option fc1_cg=2
run cg4 --option fc1_cg=4
run cg2s0 --option fc1_cg=2 --option sc1_out=0
run cg1b --option fc1_cg=1
run cg2b --option fc1_cg=2
# fc1 HBM-side fetch per launch (FETCH_SIZE, one pass each)
for v in 1 2 4; do
  PASSES="FETCH_SIZE" TAG=pmc_r4y_cg$v BENCH_ARGS="--option fc1_cg=$v" timeout -k 10 400 bash tools/pmc_pass.sh || exit 3
  python - $v <<'P'
import csv, sys, collections
v = sys.argv[1]
rows = list(csv.DictReader(open(f"gpurun_out/pmc_r4y_cg{v}/p1/run_counter_collection.csv")))
acc = collections.defaultdict(list)
for r in rows:
    if r.get("Counter_Name") == "FETCH_SIZE":
        acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
for k, vals in acc.items():
    if "7, 0, 32, 16, 4096" in k or "7, 0, 32, 16, 0, true" in k:
        print("fc1_cg", v, k[:90], "launches", len(vals), "FETCH_SIZE KB/launch (raw, x2 for wide reads)", round(sum(vals) / len(vals)))
P
done
