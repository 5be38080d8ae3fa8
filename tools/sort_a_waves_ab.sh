#!/usr/bin/env bash
# k_sort_a at one block per CU (in tree, 80 VGPRs) vs two (ab/sa8.so,
# BPE_SORT_A_WAVES=8: 64 VGPRs, 3 dwords spilled): init only, alternated
set -o pipefail
OUT=gpurun_out
: > $OUT/sort_a_waves_ab.txt
for rep in 1 2; do
  for v in tree sa8; do
    lib=""; [ $v = sa8 ] && lib=ab/sa8.so
    echo "== $v" >> $OUT/sort_a_waves_ab.txt
    BPE_LIB=$lib timeout -k 10 120 python3 tools/init_prof.py uniform 1024 >> $OUT/sort_a_waves_ab.txt 2>&1 || { echo "$v failed"; exit 1; }
  done
done
echo done
