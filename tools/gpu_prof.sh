#!/bin/bash
# rocprofv3 evidence at HEAD (trace + stats, FETCH / WRITE PMC passes keyed by stage), optional extra pytest args.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ -n "${PYTEST_ARGS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $PYTEST_ARGS -p no:cacheprovider --timeout 300 --timeout-method thread -rf > gpurun_out/pytest_extra.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_extra.log | tail -2
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
TAG=${TAG:-r3} STEPS=${STEPS:-10} bash tools/profile_round.sh
