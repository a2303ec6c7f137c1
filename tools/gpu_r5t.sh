#!/bin/bash
# Round-5 session T: MLS-style host-fed workload under a kernel + copy trace (where the wall time beyond device time goes)
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r5t"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d "$O/t" -o run --output-format csv -- \
  python3 "$R/bench.py" --workload mls --steps 4 --warmup 1 --cpu-baseline-seconds 0 --no-profile --json-out "$O/mls.json" > "$O/log" 2>&1 || { echo "trace rc=$?"; tail -5 "$O/log"; exit 1; }
python3 -c "import json; d=json.load(open('$O/mls.json')); print(d['value'], d['ms_per_step'])"
