#!/bin/bash
# gemm_bench on the transformer GEMM shapes: DIAG (no DMA / no MFMA) splits and tile variants
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 tools/bin/gemm_bench 20 ${GB_SHAPES:-qkv,fc1,fc2,o_proj} "${GB_VARS:-ref 256x128|T |128x128 8w+4ld s2|128x128 8w s2 (fc1|128x128 8w+4ld s3}" > gpurun_out/gemm_bench.log 2>&1
rc=$?; cat gpurun_out/gemm_bench.log; exit $rc
