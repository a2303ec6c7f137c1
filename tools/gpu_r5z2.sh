#!/bin/bash
# Round-5 session Z2: the adopted build (ops.hip without SLP) -- the whole GPU suite (incl. two engines alternating in
# MimiEncoder's pipeline), then the race probes under load
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r5z2"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > "$O/pytest.log" 2>&1
rc=$?; tail -3 "$O/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/race_taps.py 300 nocontrols > $O/taps.log 2>&1 || { tail -5 $O/taps.log; exit 1; }
echo "taps: $(grep -c '^loaded' $O/taps.log) of 300 loaded reps differ, $(grep -c '^idle' $O/taps.log) idle"
timeout -k 10 300 python -u tools/race_probe.py 24 all > $O/codes.log 2>&1 || { tail -5 $O/codes.log; exit 1; }
grep setting $O/codes.log
