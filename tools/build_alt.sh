#!/usr/bin/env bash
# Build a variant of the library into ab/<name>.so with extra compiler flags
# (A/B runs: BPE_LIB=ab/<name>.so).  usage: tools/build_alt.sh name -DFOO=1 ...
set -e
name=$1; shift
mkdir -p ab/build_$name
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-result -Wno-unused-value "$@" \
    -c llmtokenizer_amd/csrc/engine.hip -o ab/build_$name/engine.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ab/$name.so ab/build_$name/engine.o \
    llmtokenizer_amd/build/bpe.o llmtokenizer_amd/build/dyn_arr.o llmtokenizer_amd/build/hash_table.o -lm -ldl
echo built ab/$name.so
