#!/bin/bash
# attention V transposed reads: attn_check (error vs the f32 kernel, determinism, time) old vs new, the GPU suite's
# attention-bearing parity tests, then the engine A/B at B = 32 and B = 1
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in prev "" prev ""; do
  for bt in "32 250" "1 250" "3 100"; do
    timeout -k 10 60 tools/bin/attn_check${v:+_$v} $bt > gpurun_out/ac.log 2>&1 || { echo "attn_check $v $bt failed"; cat gpurun_out/ac.log; exit 2; }
    echo "${v:-new} $bt: $(grep 'attention_t256_h16 ' gpurun_out/ac.log | sed 's/ *attention_t256_h16 *//') $(grep 'rep 0' gpurun_out/ac.log | sed 's/.*= //;s/,.*//') $(grep -c 'differs from rep 0 in 0 halves' gpurun_out/ac.log)"
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_ragged.py -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -rf -x -q > gpurun_out/pytest_attn_tr.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_attn_tr.log
if [ $rc -ne 0 ]; then exit $rc; fi
LIBS="base new" ROUNDS=2 KEYS="attention" bash tools/ab_libs.sh || exit 3
LIBS="base new" ROUNDS=2 KEYS="attention" BENCH_ARGS="--batch 1" STEPS=50 bash tools/ab_libs.sh || exit 4
