#!/usr/bin/env bash
# TEST INFRASTRUCTURE ONLY.  Builds the unmodified reference trainer from its
# own C sources where they lie under /root/reference (read-only) into
# oracle/_ref/ (git-ignored; it travels to the GPU box like our own .so files
# so bench.py can time it as the CPU baseline).  Nothing is copied from the
# reference into the repository.
#
#   gcc -O2 <ref>/bpe/src/bpe.c <ref>/hash_table/src/hash_table.c
#       <ref>/dyn_arr/src/dyn_arr.c oracle/ref_harness.c
#       -Wl,--wrap=hash_table_merge -pthread -lm
#
# The reference has no build system; these three files
# plus libc/pthreads/libm are its whole dependency set.
set -euo pipefail
REF="${REF_ROOT:-/root/reference}"
HERE="$(cd "$(dirname "$0")" && pwd)"
OUT="$HERE/_ref"
if [ ! -f "$REF/bpe/src/bpe.c" ]; then
    echo "build_ref: reference not present at $REF; skipping" >&2
    exit 0
fi
mkdir -p "$OUT"
gcc -O2 -w \
    "$REF/bpe/src/bpe.c" "$REF/hash_table/src/hash_table.c" "$REF/dyn_arr/src/dyn_arr.c" \
    "$HERE/ref_harness.c" \
    -Wl,--wrap=hash_table_merge -pthread -lm -o "$OUT/bpe_ref"
echo "build_ref: built $OUT/bpe_ref"
