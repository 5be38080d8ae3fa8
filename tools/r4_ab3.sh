#!/usr/bin/env bash
# Round-4 A/B: the pair table as 16-byte {key, count} slots (BPE_TAB_IL=1,
# default) or two arrays (0), configs[2] and configs[3] at N=1.
set -o pipefail
OUT=${OUT:-gpurun_out}
: > $OUT/tab_il.log
for rep in 1 2; do
    for il in 1 0; do
        for m in 8192 1024; do
            echo "il=$il m=$m rep $rep" >> $OUT/tab_il.log
            BPE_TAB_IL=$il timeout -k 10 200 python3 tools/batch_check.py $m >> $OUT/tab_il.log 2>&1 || exit 1
        done
    done
done
