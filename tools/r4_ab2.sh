#!/usr/bin/env bash
# Round-4 quick A/B: init of configs[2] with pass B in groups of G tiles
# (BPE_SORT_G=16 default vs 1 = one tile per unit, the round-3 form).
set -o pipefail
OUT=${OUT:-gpurun_out}
: > $OUT/sort_g.log
for rep in 1 2; do
    for g in 16 1; do
        echo "G=$g rep $rep" >> $OUT/sort_g.log
        BPE_SORT_G=$g timeout -k 10 200 python3 tools/batch_check.py 1024 >> $OUT/sort_g.log 2>&1 || exit 1
    done
done
