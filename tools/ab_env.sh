#!/usr/bin/env bash
# A/B of environment settings on the in-tree library: ENVS="A=1 B=2;C=3" (one
# bench per ';'-separated setting, plus the default), each run twice; then
# ab/libbpe_head.so (if present) once for reference.
set -o pipefail
OUT=${OUT:-gpurun_out}
TAG=${TAG:-env}
B="python bench.py --no-encode --no-cpu-baseline"
IFS=';' read -ra SETS <<< "$ENVS"
for rep in 1 2; do
    timeout -k 10 200 $B > $OUT/ab_def_${TAG}_$rep.json 2>/dev/null || exit 1
    i=0
    for s in "${SETS[@]}"; do
        env $s timeout -k 10 200 $B > $OUT/ab_e${i}_${TAG}_$rep.json 2>/dev/null || exit 1
        i=$((i+1))
    done
done
if [ -f ab/libbpe_head.so ]; then
    BPE_LIB=ab/libbpe_head.so timeout -k 10 200 $B > $OUT/ab_head_${TAG}_1.json 2>/dev/null || exit 1
fi
echo done
