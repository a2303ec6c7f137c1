#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ragged.py tests/test_gpu_parity.py -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread -rf -x -q -k "ragged or padded or batch" > gpurun_out/pytest_rag.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_rag.log
if [ $rc -ne 0 ]; then exit $rc; fi
LIBS="base new" ROUNDS=2 STEPS=10 KEYS="qkv attention o_proj fc1 fc2 final downsample input_proj" BENCH_ARGS="--workload yodas2" bash tools/ab_libs.sh || exit 3
LIBS="base new" ROUNDS=1 STEPS=10 KEYS="qkv attention o_proj fc1 fc2 final" BENCH_ARGS="--workload mls" bash tools/ab_libs.sh || exit 4
