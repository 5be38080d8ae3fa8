#!/usr/bin/env bash
# A/B builds: ab/<name>.so = the library with extra -D flags on the HIP
# translation unit (load one with BPE_LIB=ab/<name>.so).  CPU side only.
# usage: tools/ab_build.sh <name> -DFLAG=V ...
set -e
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p ab
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-result -Wno-unused-value "$@" \
    -c llmtokenizer_amd/csrc/engine.hip -o ab/$name.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ab/$name.so ab/$name.o llmtokenizer_amd/build/bpe.o \
    llmtokenizer_amd/build/dyn_arr.o llmtokenizer_amd/build/hash_table.o -lm -ldl -lpthread
rm -f ab/$name.o
echo ab/$name.so
