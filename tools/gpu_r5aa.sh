#!/bin/bash
# Round-5 session AA: banded attention's SPLIT form (32-query workgroups, 4 waves over the key chunks) forced on the
# host-fed workloads (attn_band_split=2) vs auto (1: SPLIT only below 128 wide workgroups), alternated
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r5aa"
mkdir -p "$O"
cd "$R"
for i in 1 2; do
  for m in 2 1; do
    for w in yodas2 mls; do
      timeout -k 10 300 python -u bench.py --workload $w --steps 12 --warmup 3 --cpu-baseline-seconds 0 --option attn_band_split=$m --json-out $O/${w}_s${m}_$i.json > $O/${w}_s${m}_$i.log 2>&1 || { tail -5 $O/${w}_s${m}_$i.log; exit 1; }
      python3 -c "import json; d=json.load(open('$O/${w}_s${m}_$i.json')); s=d['stages_ms_per_step']; print('$w split=$m', d['value'], d['ms_per_step'], 'attention', s.get('attention'))"
    done
  done
done
