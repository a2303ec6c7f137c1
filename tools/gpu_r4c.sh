#!/bin/bash
# round 4: batch-1 GEMM tile / ring-depth sweep on the b1 transformer shapes
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 tools/bin/gemm_bench 20 b1_qkv,b1_fc1,b1_fc2,b1_oproj "ref 256x128 8w s3|B1 " > gpurun_out/r4c_gemm_bench_b1.log 2>&1 || { echo "gemm_bench failed"; tail -20 gpurun_out/r4c_gemm_bench_b1.log; exit 3; }
cat gpurun_out/r4c_gemm_bench_b1.log
