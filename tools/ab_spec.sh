#!/usr/bin/env bash
# A/B of the training loop: speculative graph grid splits, no speculation, and
# (if present) the library of the last commit (ab/libbpe_head.so).
set -o pipefail
OUT=${OUT:-gpurun_out}
B="python bench.py --no-encode --no-cpu-baseline"
for g in ${GRIDS:-"64,960"}; do
    BPE_SPEC_GRID=$g timeout -k 10 240 $B > $OUT/ab_spec_$g.json 2>&1 || exit 1
done
BPE_SPEC=0 timeout -k 10 240 $B > $OUT/ab_nospec.json 2>&1 || exit 1
if [ -f ab/libbpe_head.so ]; then
    BPE_LIB=ab/libbpe_head.so timeout -k 10 240 $B > $OUT/ab_head.json 2>&1 || exit 1
fi
echo done
