#!/bin/bash
# Round-5 session AB: SQ counters of the banded attention kernel alone (tools/band_bench.hip, B = 1 x 500 frames and
# B = 17 x 378): where a chunk's ~3 us go
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r5ab"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
i=0
for G in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT" \
         "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $G --kernel-trace -d "$O/p$i" -o run --output-format csv -- "$R/ab/band_bench" 1 500 17 378 \
    > "$O/p$i.log" 2>&1 || { echo "pass $i failed rc=$?"; tail -20 "$O/p$i.log"; exit 1; }
  echo "pass $i ok"
done
