#!/bin/bash
# Round-5 session AF: ticket words written inside the graph (set_io passes the pinned destinations) -- GPU suite,
# batch-1 trace, then batch 1 / B = 32 alternated against the library before the ticket change (ab/libmimi_hip_head.so)
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r5af"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > "$O/pytest.log" 2>&1
rc=$?; tail -2 "$O/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 bash tools/trace_b1.sh > $O/trace_b1.log 2>&1 || { tail -5 $O/trace_b1.log; exit 1; }
head -3 $O/trace_b1.log
for i in 1 2 3; do
  for v in new head; do
    if [ $v = head ]; then export MIMI_HIP_LIB=$R/ab/libmimi_hip_head.so; else unset MIMI_HIP_LIB; fi
    timeout -k 10 200 python -u bench.py --batch 1 --steps 60 --cpu-baseline-seconds 0 --no-f32-mode --json-out $O/b1_${v}_$i.json > $O/b1_${v}_$i.log 2>&1 || { tail -5 $O/b1_${v}_$i.log; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b1_${v}_$i.json')); print('b1 $v', d['value'], d['ms_per_step'])"
  done
done
unset MIMI_HIP_LIB
timeout -k 10 200 python -u bench.py --steps 20 --cpu-baseline-seconds 0 --no-f32-mode --json-out $O/b32_new.json > $O/b32_new.log 2>&1 || { tail -5 $O/b32_new.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/b32_new.json')); print('b32 new', d['value'], d['ms_per_step'], d['b1_k8_pipelined']['value'], d['per_utterance_k32']['value'])"
