#!/bin/bash
# Round-5 session AI: the chain's flag + granules zeroed by set_io_kernel before each replay (no memset node) --
# GPU suite, batch-1 trace, B = 32 bench
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r5ai"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > "$O/pytest.log" 2>&1
rc=$?; tail -2 "$O/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 bash tools/trace_b1.sh > $O/trace_b1.log 2>&1 || { tail -5 $O/trace_b1.log; exit 1; }
head -3 $O/trace_b1.log
K=32 timeout -k 10 400 bash tools/trace_b1.sh > $O/trace_b1_k32.log 2>&1 || { tail -5 $O/trace_b1_k32.log; exit 1; }
head -3 $O/trace_b1_k32.log
timeout -k 10 200 python -u bench.py --steps 20 --cpu-baseline-seconds 0 --no-f32-mode --json-out $O/b32.json > $O/b32.log 2>&1 || { tail -5 $O/b32.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/b32.json')); print('b32', d['value'], d['ms_per_step'], d['b1_k8']['value'], d['b1_k8_pipelined']['value'], d['per_utterance_k32']['value'])"
