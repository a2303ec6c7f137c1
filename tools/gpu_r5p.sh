#!/bin/bash
# Round-5 session P: headline loop with one-behind waits (bench.py) vs each step waited (HEAD's bench, tools/bench_sync_ref.py)
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r5p2"
mkdir -p "$O"
cd "$R"
for i in 1 2; do
  for v in new old; do
    B=bench.py; [ $v = old ] && B=tools/bench_sync_ref.py
    timeout -k 10 300 python -u $B --steps 20 --cpu-baseline-seconds 0 --no-f32-mode --json-out $O/b32_${v}_$i.json > $O/b32_${v}_$i.log 2>&1 || { tail -5 $O/b32_${v}_$i.log; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b32_${v}_$i.json')); print('b32 $v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['roofline'].get('timing'), 'b1_k8', d['b1_k8']['value'], 'b1p', d.get('b1_k8_pipelined',{}).get('value'), 's8d', d['s8d_h2d_to_d2h']['value'], 'k32', d['k32']['value'], 'utt', d['per_utterance_k32']['value'])"
  done
done
