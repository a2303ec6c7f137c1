#!/bin/bash
# Round-5 session N: per-utterance loop under kernel + copy + HIP API trace (this build)
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r5n"
mkdir -p "$O"
unset MIMI_HIP_LIB
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-trace -d "$O/t" -o run --output-format csv -- \
  python3 "$R/tools/trace_utt.py" run 12 > "$O/traced.log" 2>&1 || { echo "trace rc=$?"; tail -5 "$O/traced.log"; exit 1; }
tail -1 "$O/traced.log"; ls "$O/t"
