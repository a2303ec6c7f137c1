set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
(cat /sys/fs/cgroup/cpu.max 2>/dev/null; nproc; python -c "import os;print(len(os.sched_getaffinity(0)))"; echo OMP=$OMP_NUM_THREADS) > gpurun_out/cpuinfo.txt 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -3
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -5 gpurun_out/smoke.log; exit 3; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_b32.json > gpurun_out/bench.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench.log; exit 4; }
tail -c 600 gpurun_out/bench_b32.json
