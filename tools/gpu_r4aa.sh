#!/bin/bash
# round 4: stage-1 block as two 4-wave workgroups per CU (engine option res1_form = 1): parity and A/B
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_res1_form.py \
  "tests/test_gpu_parity.py::test_kernel_options_identical_codes" > gpurun_out/r4aa_pytest.log 2>&1 || { echo "pytest failed"; grep -E "Error|assert" gpurun_out/r4aa_pytest.log | head; tail -5 gpurun_out/r4aa_pytest.log; exit 1; }
tail -1 gpurun_out/r4aa_pytest.log
run() {  # tag, bench args...
  local tag=$1; shift
  timeout -k 10 300 python -u bench.py "$@" --cpu-baseline-seconds 0 --no-f32-mode --pmc-pass --json-out gpurun_out/r4aa_$tag.json > gpurun_out/r4aa_$tag.log 2>&1 || { echo "bench $tag failed"; tail -30 gpurun_out/r4aa_$tag.log; exit 2; }
  python - $tag <<'P'
import json,sys; t=sys.argv[1]; d=json.load(open(f"gpurun_out/r4aa_{t}.json"))
st=d["stages_ms_per_step"]
print(t, d["value"], d["ms_per_step"], {k: st.get(k) for k in ("res_s1","res_down_s0","down_s1")})
P
}
run f0 --option res1_form=0
run f1 --option res1_form=1
run f0b --option res1_form=0
run f1b --option res1_form=1
