#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ragged.py tests/test_gpu_parity.py tests/test_stage0_fused.py tests/test_pipeline_gpu.py -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -rf -x -q > gpurun_out/pytest_pack.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_pack.log
if [ $rc -ne 0 ]; then exit $rc; fi
LIBS="base new" ROUNDS=2 STEPS=10 KEYS="layernorm qkv attention o_proj fc1 fc2 downsample" BENCH_ARGS="--workload yodas2" bash tools/ab_libs.sh || exit 3
LIBS="base new" ROUNDS=2 STEPS=10 KEYS="layernorm qkv attention o_proj fc1 fc2" BENCH_ARGS="--workload mls" bash tools/ab_libs.sh || exit 4
