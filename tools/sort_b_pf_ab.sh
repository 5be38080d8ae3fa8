#!/usr/bin/env bash
# k_sort_b with the next chunk's loads in flight (ab/sbpf.so, 64 VGPRs) vs in
# tree (56): init only, uniform and english-like 1 GiB, alternated
set -o pipefail
OUT=gpurun_out
: > $OUT/sort_b_pf_ab.txt
for rep in 1 2; do
  for v in tree sbpf; do
    lib=""; [ $v = sbpf ] && lib=ab/sbpf.so
    echo "== $v" >> $OUT/sort_b_pf_ab.txt
    BPE_LIB=$lib timeout -k 10 120 python3 tools/init_prof.py uniform 1024 >> $OUT/sort_b_pf_ab.txt 2>&1 || { echo "$v failed"; exit 1; }
  done
done
echo done
