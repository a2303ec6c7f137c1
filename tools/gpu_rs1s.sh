#!/bin/bash
# res_s1 LDS swizzle: stage-1 / ragged / stage-0 parity tests, then an A/B against the HEAD build
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_ragged.py tests/test_stage0_fused.py -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -rf -x -q > gpurun_out/pytest_rs1s.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_rs1s.log
if [ $rc -ne 0 ]; then exit $rc; fi
LIBS="base new" ROUNDS=3 KEYS="res_s1 res_down_s0" bash tools/ab_libs.sh || exit 3
