#!/bin/bash
# builds tools/bin/libmimi_hip_rr{1,2,4}.so: the engine with resblock_rows.hip compiled under RR_DIAG (timing only)
set -eu
cd "$(dirname "$0")/../tokenize-audio_amd/csrc"
mkdir -p ../../tools/bin build_qa
OBJS="build/gemm.hip.o build/qkv_attn.hip.o build/resblock.hip.o build/stage0_fused.hip.o build/ops.hip.o build/resample.hip.o build/bpe.hip.o build/engine.cpp.o build/flac.cpp.o build/safetensors.cpp.o"
for D in 1 2 4; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-result --offload-arch=gfx950 -DRR_DIAG=$D -c resblock_rows.hip -o build_qa/rr$D.o
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../../tools/bin/libmimi_hip_rr$D.so $OBJS build_qa/rr$D.o
done
