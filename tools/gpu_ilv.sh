#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 tools/bin/gemm_bench 20 down_s1,down_s2,down_s3 "ref 256x128|pair PERSIST 8w+4ld s2|pair PERSIST DIAG nomma|256x128 8w+4ld s3" > gpurun_out/gb_ilv1.log 2>&1 || { cat gpurun_out/gb_ilv1.log; exit 2; }
timeout -k 10 300 tools/bin/gemm_bench 20 qkv,fc1,fc2,res3_s2 "ref 256x128|T 128x128 8w+4ld s2|T 128x128 8w+4ld s3|256x128 8w+4ld s3|128x128 8w+4ld s2|128x128 8w+4ld s3" > gpurun_out/gb_ilv2.log 2>&1 || { cat gpurun_out/gb_ilv2.log; exit 3; }
cat gpurun_out/gb_ilv1.log gpurun_out/gb_ilv2.log
