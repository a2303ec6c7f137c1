#!/bin/bash
# Round-5 session L: decomposition-invariant banded attention -- its tests, the GPU suite, then per-utterance and
# MLS-style timing against the previous build (ab/libmimi_hip_band0.so)
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r5l"
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_attention_band.py > "$O/pytest_band.log" 2>&1
rc=$?; tail -3 "$O/pytest_band.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests > "$O/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$O/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export MIMI_HIP_LIB=$R/ab/libmimi_hip_band0.so; else unset MIMI_HIP_LIB; fi
    timeout -k 10 200 python3 -u tools/trace_utt.py run 24 > "$O/utt_${v}_$i.log" 2>&1 || { tail -5 "$O/utt_${v}_$i.log"; exit 1; }
    echo "utt $v: $(tail -1 $O/utt_${v}_$i.log)"
    timeout -k 10 200 python -u bench.py --workload mls --steps 3 --warmup 1 --cpu-baseline-seconds 0 --json-out $O/mls_${v}_$i.json > $O/mls_${v}_$i.log 2>&1 || { tail -5 $O/mls_${v}_$i.log; exit 1; }
    python3 -c "import json; d=json.load(open('$O/mls_${v}_$i.json')); s=d['stages_ms_per_step']; print('mls $v', d['value'], d['ms_per_step'], 'attention', s.get('attention'))"
  done
done
