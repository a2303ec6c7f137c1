#!/bin/bash
# Round-5 session Q: headline timed region eager + light events (default) vs hipGraph replays without events (--no-profile)
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r5q"
mkdir -p "$O"
cd "$R"
for i in 1 2 3; do
  for v in light graph; do
    X=""; [ $v = graph ] && X="--no-profile"
    timeout -k 10 300 python -u bench.py --steps 30 --cpu-baseline-seconds 0 --no-f32-mode --pmc-pass $X --json-out $O/b32_${v}_$i.json > $O/b32_${v}_$i.log 2>&1 || { tail -5 $O/b32_${v}_$i.log; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b32_${v}_$i.json')); print('b32 $v', d['value'], d['ms_per_step'], 'graph_replays', d.get('graph_replays'))"
  done
done
