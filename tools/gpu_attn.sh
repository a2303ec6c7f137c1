#!/bin/bash
# attention rewrite check: accuracy / timing probe, the parity suites, then base-vs-new bench A/B at B = 32 and B = 1
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for bt in "32 250" "1 250" "8 250" "16 250" "3 100" "2 1"; do
  timeout -k 10 60 tools/bin/attn_check $bt > gpurun_out/attn_check_${bt// /_}.log 2>&1 || { echo "attn_check $bt failed"; cat gpurun_out/attn_check_${bt// /_}.log; exit 2; }
  echo "== $bt"; cat gpurun_out/attn_check_${bt// /_}.log
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_ragged.py tests/test_stage0_fused.py -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -rf -x -q > gpurun_out/pytest_attn.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_attn.log
if [ $rc -ne 0 ]; then exit $rc; fi
LIBS="base new" ROUNDS=2 KEYS="qkv attention layernorm fc1" bash tools/ab_libs.sh || exit 3
LIBS="base new" ROUNDS=2 KEYS="qkv attention layernorm fc1" BENCH_ARGS="--batch 1" bash tools/ab_libs.sh || exit 4
