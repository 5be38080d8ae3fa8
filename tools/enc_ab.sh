#!/usr/bin/env bash
# Encode A/B: the 32k-merge list trained once, then the 10 GiB encode with the
# in-tree library and each ab/*.so given in LIBS, twice each.
set -o pipefail
OUT=${OUT:-gpurun_out}
TAG=${TAG:-enc}
timeout -k 10 120 python3 tools/enc_prof.py train > $OUT/encab_$TAG.log 2>&1 || exit 1
for rep in 1 2; do
    echo "new $rep" >> $OUT/encab_$TAG.log
    timeout -k 10 120 python3 tools/enc_prof.py enc >> $OUT/encab_$TAG.log 2>&1 || exit 1
    for l in $LIBS; do
        echo "$l $rep" >> $OUT/encab_$TAG.log
        BPE_LIB=$l timeout -k 10 120 python3 tools/enc_prof.py enc >> $OUT/encab_$TAG.log 2>&1 || exit 1
    done
done
echo done
