#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ragged.py tests/test_gpu_parity.py -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -rf -x -q -k "ragged or padded or chunks" > gpurun_out/pytest_pack.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_pack.log
if [ $rc -ne 0 ]; then exit $rc; fi
for v in base new base new; do
  if [ $v = new ]; then unset MIMI_HIP_LIB; else export MIMI_HIP_LIB=$GRAFT_REPO_ROOT/tools/bin/libmimi_hip_$v.so; fi
  echo -n "$v: "; timeout -k 10 300 python tools/mls_probe.py 320 10 20 2>/dev/null | tail -1 || exit 2
done
unset MIMI_HIP_LIB
LIBS="base new" ROUNDS=1 STEPS=10 KEYS="qkv fc1" BENCH_ARGS="--workload mls" bash tools/ab_libs.sh || exit 4
LIBS="base new" ROUNDS=1 STEPS=10 KEYS="qkv fc1" BENCH_ARGS="--workload yodas2" bash tools/ab_libs.sh || exit 4
