#!/bin/bash
# round 4: SQ counters of the fused q/k/v + attention kernel (and its QA_DIAG MFMA-only build)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
P="SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,GRBM_GUI_ACTIVE;SQ_WAVE_CYCLES,SQ_WAIT_INST_LDS,SQ_VALU_MFMA_BUSY_CYCLES,SQ_LDS_BANK_CONFLICT,GRBM_GUI_ACTIVE"
PASSES="$P" TAG=pmc_sq_r4n bash tools/pmc_pass.sh || exit 1
python tools/sq_table.py pmc_sq_r4n > gpurun_out/r4n_sq.txt || exit 2
MIMI_HIP_LIB=$PWD/tools/bin/libmimi_hip_qa3.so PASSES="$P" TAG=pmc_sq_r4n_d3 bash tools/pmc_pass.sh || exit 3
python tools/sq_table.py pmc_sq_r4n_d3 > gpurun_out/r4n_sq_d3.txt || exit 4
grep -E "kernel|qkv_attention|fc1|fc2|o_proj|gemm_planes_kernel<128" gpurun_out/r4n_sq.txt | head -12
grep -E "kernel|qkv_attention" gpurun_out/r4n_sq_d3.txt | head -4
