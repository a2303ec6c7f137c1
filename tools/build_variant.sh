#!/bin/bash
# A/B library builds: ab/libmimi_hip_NAME.so = the in-tree objects (tokenize-audio_amd/csrc/build, `make` first) with
# one source recompiled with extra flags, e.g.
#   bash tools/build_variant.sh r1s_d3 res1_stream.hip "-DMIMI_R1S_DEPTH2=3"
# (the flags are the Makefile's device flags: no packed f32, -ffp-contract=off).  ab/ travels to the GPU box.
set -eu
NAME=$1; SRC=$2; DEFS=${3:-}
R="$(cd "$(dirname "$0")/.." && pwd)"
C="$R/tokenize-audio_amd/csrc"
T=$(mktemp -d)
EXTRA=""
case "$SRC" in stage0_fused.hip|ops.hip) EXTRA="-fno-slp-vectorize" ;; engine.cpp) EXTRA="-x hip" ;; esac
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-result --offload-arch=gfx950 \
  -Xclang -target-feature -Xclang -packed-fp32-ops $EXTRA $DEFS -c "$C/$SRC" -o "$T/$SRC.o" 2> >(grep -v "not a recognized feature" >&2)
OBJS=$(ls "$C"/build/*.o | grep -v "/$SRC.o$")
mkdir -p "$R/ab"
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$R/ab/libmimi_hip_$NAME.so" $OBJS "$T/$SRC.o"
rm -rf "$T"
echo "ab/libmimi_hip_$NAME.so"
