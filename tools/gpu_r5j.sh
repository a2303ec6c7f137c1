#!/bin/bash
# Round-5 session J: per-utterance loop (encode_audio_chunk, K = 32) untraced, then under a kernel + copy trace
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r5j"
mkdir -p "$O"
timeout -k 10 200 python3 -u "$R/tools/trace_utt.py" run 24 > "$O/untraced.log" 2>&1 || { tail -5 "$O/untraced.log"; exit 1; }
tail -1 "$O/untraced.log"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d "$O/t" -o run --output-format csv -- \
  python3 "$R/tools/trace_utt.py" run 24 > "$O/traced.log" 2>&1 || { echo "trace rc=$?"; tail -5 "$O/traced.log"; exit 1; }
tail -1 "$O/traced.log"
python3 "$R/tools/trace_utt.py" summary "$O/t" > "$O/summary.txt" && cat "$O/summary.txt"
