#!/bin/bash
# rocprofv3 kernel trace of the batch-1 bench (graph replays on), summarised per encode step
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/trace_b${B:-1}_k${K:-8}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/t" -o run --output-format csv -- \
  python3 "$R/bench.py" --batch ${B:-1} --num-quantizers ${K:-8} --steps 30 --warmup 5 --cpu-baseline-seconds 0 --no-f32-mode --no-profile \
  > "$OUT/log" 2>&1 || { echo "trace failed rc=$?"; tail -20 "$OUT/log"; exit 1; }
python3 "$R/tools/trace_summary.py" "$OUT/t" > "$OUT/summary.txt" && cat "$OUT/summary.txt"
