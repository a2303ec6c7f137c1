#!/bin/bash
# round-3 evidence at HEAD: rocprofv3 trace + stats + FETCH/WRITE PMC (profile_round.sh), then the SQ/GRBM passes
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r3f} STEPS=10 bash tools/profile_round.sh || exit 1
PASSES="SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,GRBM_GUI_ACTIVE;SQ_WAVE_CYCLES,SQ_WAIT_INST_LDS,SQ_VALU_MFMA_BUSY_CYCLES,SQ_LDS_BANK_CONFLICT,GRBM_GUI_ACTIVE" TAG=pmc_sq_${TAG:-r3f} bash tools/pmc_pass.sh || exit 2
