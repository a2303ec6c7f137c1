#!/bin/bash
# builds tools/bin/libmimi_hip_s0p{1,2,3}.so: the engine with stage0_fused.hip compiled under S0F_PRIO=N (the block
# waves raise their issue priority over the conv waves; a scheduling hint, the same bits) -- for A/B timing
set -eu
cd "$(dirname "$0")/../tokenize-audio_amd/csrc"
mkdir -p ../../tools/bin build_qa
OBJS="build/gemm.hip.o build/qkv_attn.hip.o build/oproj_ln.hip.o build/resblock_rows.hip.o build/resblock.hip.o build/ops.hip.o build/resample.hip.o build/bpe.hip.o build/engine.cpp.o build/flac.cpp.o build/safetensors.cpp.o"
for V in ${PRIO_LIST:-1 2 3}; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-result --offload-arch=gfx950 -fno-slp-vectorize -DS0F_PRIO=$V -c stage0_fused.hip -o build_qa/s0p$V.o &
done
wait
for V in ${PRIO_LIST:-1 2 3}; do
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../../tools/bin/libmimi_hip_s0p$V.so $OBJS build_qa/s0p$V.o
done
