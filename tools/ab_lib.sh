#!/usr/bin/env bash
# A/B of the training loop: the in-tree library against ab/libbpe_head.so (and
# ab/libbpe_alt.so if present), alternated twice; then the block timeline of
# the in-tree library.
set -o pipefail
OUT=${OUT:-gpurun_out}
TAG=${TAG:-ab}
B="python bench.py --no-encode --no-cpu-baseline"
for rep in 1 2; do
    timeout -k 10 200 $B > $OUT/ab_new_${TAG}_$rep.json 2>/dev/null || exit 1
    BPE_LIB=ab/libbpe_head.so timeout -k 10 200 $B > $OUT/ab_head_${TAG}_$rep.json 2>/dev/null || exit 1
    if [ -n "$ALT_ENV" ]; then
        env $ALT_ENV timeout -k 10 200 $B > $OUT/ab_altenv_${TAG}_$rep.json 2>/dev/null || exit 1
    fi
    if [ -f ab/libbpe_alt.so ]; then
        BPE_LIB=ab/libbpe_alt.so timeout -k 10 200 $B > $OUT/ab_alt_${TAG}_$rep.json 2>/dev/null || exit 1
    fi
done
if [ -n "$SHARDED" ]; then
    timeout -k 10 200 $B --sharded > $OUT/ab_shnew_${TAG}.json 2>/dev/null || exit 1
    BPE_LIB=ab/libbpe_head.so timeout -k 10 200 $B --sharded > $OUT/ab_shhead_${TAG}.json 2>/dev/null || exit 1
fi
BPE_DEBUG_TS=1 timeout -k 10 200 $B > $OUT/ab_ts_${TAG}.json 2> $OUT/ab_ts_${TAG}.err || exit 1
echo done
