#!/bin/bash
# Round-5 session M: host path with pinned staging + polled waits vs HEAD (ab/libmimi_hip_band1.so): tests, then the
# per-utterance loop and the B = 32 bench alternated
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r5m"
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_encode_host.py tests/test_gpu_parity.py -k "host or chain or chunk or async or thread" > "$O/pytest.log" 2>&1
rc=$?; tail -2 "$O/pytest.log"; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export MIMI_HIP_LIB=$R/ab/libmimi_hip_band1.so; else unset MIMI_HIP_LIB; fi
    timeout -k 10 200 python3 -u tools/trace_utt.py host > "$O/utt_${v}_$i.log" 2>&1 || { tail -5 "$O/utt_${v}_$i.log"; exit 1; }
    echo "utt $v: $(tail -1 $O/utt_${v}_$i.log)"
    timeout -k 10 200 python -u bench.py --steps 20 --cpu-baseline-seconds 0 --no-f32-mode --json-out $O/b32_${v}_$i.json > $O/b32_${v}_$i.log 2>&1 || { tail -5 $O/b32_${v}_$i.log; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b32_${v}_$i.json')); print('b32 $v', d['value'], d['ms_per_step'], 'b1_k8', d['b1_k8']['value'], 'utt', d['per_utterance_k32']['value'], 's8d', d['s8d_h2d_to_d2h']['value'])"
  done
done
