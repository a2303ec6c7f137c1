#!/bin/bash
# rocprofv3 evidence for the bench: kernel trace + stats, then FETCH_SIZE and WRITE_SIZE in separate PMC
# passes (never combined with runtime/sys tracing).  Each step under its own time limit; stop on failure.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${TAG:-r1}
OUT="$R/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH="$R/bench.py"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
  python3 "$BENCH" --steps ${STEPS:-10} --warmup 3 --cpu-baseline-seconds 0 --json-out "$OUT/bench_under_trace.json" \
  --dump-sequence "$OUT/stage_sequence.json" --pmc-pass \
  > "$OUT/trace.log" 2>&1 || { echo "trace failed rc=$?"; tail -20 "$OUT/trace.log"; exit 1; }
echo "trace ok"
if [ "${PMC:-1}" = 1 ]; then
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 600 rocprofv3 --pmc $C --kernel-trace -d "$OUT/pmc_$C" -o run --output-format csv -- \
      python3 "$BENCH" --steps 2 --warmup 1 --cpu-baseline-seconds 0 --no-profile --pmc-pass \
      > "$OUT/pmc_$C.log" 2>&1 || { echo "pmc $C failed rc=$?"; tail -20 "$OUT/pmc_$C.log"; exit 1; }
    echo "pmc $C ok"
  done
fi
find "$OUT" -name "*.csv" | head -20
