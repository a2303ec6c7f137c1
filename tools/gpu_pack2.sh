#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
LIBS="base new" ROUNDS=2 STEPS=10 KEYS="layernorm qkv attention o_proj fc1 fc2" BENCH_ARGS="--workload yodas2" bash tools/ab_libs.sh || exit 3
LIBS="base new" ROUNDS=2 STEPS=10 KEYS="layernorm qkv attention o_proj fc1 fc2" BENCH_ARGS="--workload mls" bash tools/ab_libs.sh || exit 4
