#!/bin/bash
# builds tools/bin/libmimi_hip_qa{1,3,5}.so: the engine with qkv_attn.hip compiled under QA_DIAG (timing only)
set -eu
cd "$(dirname "$0")/../tokenize-audio_amd/csrc"
mkdir -p ../../tools/bin build_qa
OBJS="build/gemm.hip.o build/resblock.hip.o build/stage0_fused.hip.o build/ops.hip.o build/resample.hip.o build/bpe.hip.o build/engine.cpp.o build/flac.cpp.o build/safetensors.cpp.o"
for D in 1 8 16 24; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-result --offload-arch=gfx950 -DQA_DIAG=$D -c qkv_attn.hip -o build_qa/qa$D.o
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../../tools/bin/libmimi_hip_qa$D.so $OBJS build_qa/qa$D.o
done
