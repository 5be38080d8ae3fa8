#!/usr/bin/env bash
# configs[1] A/B: the tree's library against ab/<name>.so variants, alternated
# twice (tools/c1_ab2.py), then the tree's per-merge timeline.  LIBS="a b ..."
set -o pipefail
OUT=${OUT:-gpurun_out}
cd ${GRAFT_REPO_ROOT:-.}
: > $OUT/c1_ab2.txt
for rep in 1 2; do
  for L in tree $LIBS; do
    if [ "$L" = tree ]; then
      timeout -k 10 120 python -u tools/c1_ab2.py 7 >> $OUT/c1_ab2.txt 2>$OUT/c1_ab2.err || { tail $OUT/c1_ab2.err; exit 1; }
    else
      BPE_LIB=ab/$L.so timeout -k 10 120 python -u tools/c1_ab2.py 7 >> $OUT/c1_ab2.txt 2>$OUT/c1_ab2.err || { tail $OUT/c1_ab2.err; exit 1; }
    fi
  done
done
cat $OUT/c1_ab2.txt
BPE_DEBUG=1 BPE_DEBUG_TS=1 timeout -k 10 120 python -u tools/c1_prof.py > $OUT/c1_ts2.txt 2>&1 || { tail $OUT/c1_ts2.txt; exit 1; }
grep -h "timeline\|select phases" $OUT/c1_ts2.txt | cut -c1-900
