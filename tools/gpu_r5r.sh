#!/bin/bash
# Round-5 session R: persistent RVQ chain with the candidates' code rows staged in LDS by LDS-DMA (one round trip) vs
# HEAD (ab/libmimi_hip_rvq0.so): quantizer / chain tests, then per-utterance K = 32 and batch-1 K = 32 timing
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r5r"
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_parity.py tests/test_encode_host.py -k "quantizer or chain or rvq or host or golden" > "$O/pytest.log" 2>&1
rc=$?; tail -2 "$O/pytest.log"; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export MIMI_HIP_LIB=$R/ab/libmimi_hip_rvq0.so; else unset MIMI_HIP_LIB; fi
    timeout -k 10 200 python3 -u tools/trace_utt.py host > "$O/utt_${v}_$i.log" 2>&1 || { tail -5 "$O/utt_${v}_$i.log"; exit 1; }
    echo "utt $v: $(tail -1 $O/utt_${v}_$i.log)"
    timeout -k 10 200 python -u bench.py --batch 1 --num-quantizers 32 --steps 30 --warmup 3 --cpu-baseline-seconds 0 --no-f32-mode --json-out $O/b1k32_${v}_$i.json > $O/b1k32_${v}_$i.log 2>&1 || { tail -5 $O/b1k32_${v}_$i.log; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b1k32_${v}_$i.json')); s=d['stages_ms_per_step']; print('b1 k32 $v', d['value'], d['ms_per_step'], 'rvq', s.get('rvq'))"
  done
done
