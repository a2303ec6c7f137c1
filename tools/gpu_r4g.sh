#!/bin/bash
# round 4: full GPU test suite at HEAD, then batch-1 kernel traces (K = 8 and K = 32)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r4g_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r4g_pytest.log; exit 1; }
tail -3 gpurun_out/r4g_pytest.log
K=8 bash tools/trace_b1.sh || exit 2
K=32 bash tools/trace_b1.sh || exit 3
