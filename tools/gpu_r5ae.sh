#!/bin/bash
# Round-5 session AE: ticket words written by one kernel (ticket_out) instead of two D2H copies -- GPU suite, then
# batch 1 / 4 and B = 32 alternated against HEAD's library (ab/libmimi_hip_head.so)
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r5ae"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > "$O/pytest.log" 2>&1
rc=$?; tail -2 "$O/pytest.log"; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in new head; do
    if [ $v = head ]; then export MIMI_HIP_LIB=$R/ab/libmimi_hip_head.so; else unset MIMI_HIP_LIB; fi
    for spec in "b1:--batch 1 --steps 40" "b4:--batch 4 --steps 30" "b32:--steps 20"; do
      n=${spec%%:*}; a=${spec#*:}
      timeout -k 10 200 python -u bench.py $a --cpu-baseline-seconds 0 --no-f32-mode --json-out $O/${n}_${v}_$i.json > $O/${n}_${v}_$i.log 2>&1 || { tail -5 $O/${n}_${v}_$i.log; exit 1; }
      python3 -c "import json; d=json.load(open('$O/${n}_${v}_$i.json')); print('$n $v', d['value'], d['ms_per_step'], d.get('b1_k8_pipelined', {}).get('value'), d.get('per_utterance_k32', {}).get('value'))"
    done
  done
done
