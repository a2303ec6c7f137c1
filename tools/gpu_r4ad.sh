#!/bin/bash
# round 4 evidence at HEAD (res1_form = 1): full GPU test suite, then tools/gpu_r4ev.sh (rocprofv3 trace + stats + PMC,
# SQ passes, bench lines, smoke) under TAG r4ad
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r4ad_pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|assert" gpurun_out/r4ad_pytest_gpu.log | head; tail -5 gpurun_out/r4ad_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r4ad_pytest_gpu.log
TAG=r4ad bash tools/gpu_r4ev.sh
