#!/bin/bash
# Round-5 evidence session: the GPU suite, smoke, the headline bench, rocprofv3 trace + PMC bytes, SQ passes, the
# drop-in workloads.  Every GPU step under its own limit; stop at the first crash / timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r5f}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error" $O/pytest_gpu.log | head; exit $rc; fi
cp gpurun_out/parity_report.json $O/parity_report.json 2>/dev/null
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py --json-out $O/bench_b32.json > $O/bench_b32.log 2>&1 || { echo bench failed; tail $O/bench_b32.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_b32.json')); print('b32', d['value'], d['ms_per_step'], d['roofline']['frac'], d['s8d_h2d_to_d2h']['value'])"
TAG=$TAG STEPS=10 timeout -k 10 900 bash tools/profile_round.sh > $O/profile_round.log 2>&1 || { echo profile failed; tail $O/profile_round.log; exit 1; }
echo profile ok
PASSES="SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_WAIT_INST_LDS,GRBM_GUI_ACTIVE;SQ_VALU_MFMA_BUSY_CYCLES,SQ_LDS_BANK_CONFLICT,GRBM_GUI_ACTIVE" TAG=${TAG}_sq timeout -k 10 400 bash tools/pmc_pass.sh > $O/sq.log 2>&1 || { echo sq failed; tail $O/sq.log; exit 1; }
echo sq ok
for spec in "b1:--batch 1 --no-f32-mode" "b4:--batch 4 --no-f32-mode" "yodas2:--workload yodas2 --steps 12 --warmup 2" "mls:--workload mls --steps 8 --warmup 1"; do
  name=${spec%%:*}; args=${spec#*:}
  timeout -k 10 300 python -u bench.py --cpu-baseline-seconds 0 $args --json-out $O/bench_$name.json > $O/bench_$name.log 2>&1 || { echo "$name failed"; tail -5 $O/bench_$name.log; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$name.json')); print('$name', d['value'], d['ms_per_step'])"
done
