#!/bin/bash
# round 4: full GPU test suite at HEAD
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r4x_pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|assert" gpurun_out/r4x_pytest_gpu.log | head; tail -5 gpurun_out/r4x_pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r4x_pytest_gpu.log
