#!/bin/bash
# One rocprofv3 PMC pass per counter group over a short bench (kernel trace + counters only).
#   PASSES="SQ_WAVE_CYCLES,SQ_BUSY_CYCLES;SQ_LDS_BANK_CONFLICT" TAG=x bash tools/pmc_pass.sh
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${TAG:-pmc}
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
IFS=';' read -ra GROUPS_ <<< "$PASSES"
for G in "${GROUPS_[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc ${G//,/ } --kernel-trace -d "$OUT/p$i" -o run --output-format csv -- \
    python3 "$R/bench.py" --steps 2 --warmup 1 --cpu-baseline-seconds 0 --no-profile --pmc-pass ${BENCH_ARGS:-} \
    > "$OUT/p$i.log" 2>&1 || { echo "pass $i ($G) failed rc=$?"; tail -20 "$OUT/p$i.log"; exit 1; }
  echo "pass $i ok: $G"
done
