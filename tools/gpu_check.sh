#!/bin/bash
# GPU parity tests, then bench lines at B = 32 (headline, with the f32-mode and stage profile) and B = 1 / 4
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out
STEP_BENCH=0 bash tools/gpu_round.sh || exit 1
timeout -k 10 300 python bench.py --cpu-baseline-seconds 0 ${B32_ARGS:-} > gpurun_out/bench32.log 2>&1 || { echo bench32 failed; tail gpurun_out/bench32.log; exit 1; }
tail -1 gpurun_out/bench32.log | cut -c1-300
for B in ${SMALL_BATCHES:-1 4}; do
  timeout -k 10 300 python bench.py --batch $B --cpu-baseline-seconds 0 --no-f32-mode --steps 50 --warmup 10 > gpurun_out/bench$B.log 2>&1 || { echo bench$B failed; tail gpurun_out/bench$B.log; exit 1; }
  tail -1 gpurun_out/bench$B.log | cut -c1-200
done
