#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_ragged.py tests/test_stage0_fused.py -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -rf -x -q > gpurun_out/pytest_rs1.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_rs1.log
if [ $rc -ne 0 ]; then exit $rc; fi
LIBS="base new" ROUNDS=3 KEYS="res_s1" bash tools/ab_libs.sh || exit 3
LIBS="base new" ROUNDS=1 KEYS="res_s1" BENCH_ARGS="--batch 1" bash tools/ab_libs.sh || exit 4
