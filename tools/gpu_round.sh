#!/bin/bash
# One GPU-box session: parity tests, then the bench (each step under its own time limit; stop on a
# crash/abort/timeout, continue past ordinary test failures).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEP_TESTS=${STEP_TESTS:-1}
STEP_BENCH=${STEP_BENCH:-1}
if [ "$STEP_TESTS" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf > gpurun_out/pytest_gpu.log 2>&1
  rc=$?
  echo "pytest exit $rc"; grep -E "PASS|FAIL|ERROR" gpurun_out/pytest_gpu.log | tail -60
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
fi
if [ "$STEP_BENCH" = 1 ]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
  rc=$?
  echo "bench exit $rc"; tail -3 gpurun_out/bench.log
  exit $rc
fi
