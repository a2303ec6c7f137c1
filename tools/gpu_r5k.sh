#!/bin/bash
# Round-5 session K: mimi_encode_host tests, then the per-utterance loop timed and traced again
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r5k"
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_encode_host.py tests/test_gpu_parity.py -k "host or chain or chunk" > "$O/pytest.log" 2>&1
rc=$?; tail -3 "$O/pytest.log"; [ $rc -eq 0 ] || exit $rc
bash "$R/tools/gpu_r5j.sh" && cp -r "$R/gpurun_out/r5j" "$O/trace"
