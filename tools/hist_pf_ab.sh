#!/usr/bin/env bash
# count pass with the next round's loads in flight (in-tree, BPE_HIST_PF=1) vs without
# (ab/pf0.so), inside the real init of 16 / 8192 / 1024-merge jobs
set -o pipefail
OUT=gpurun_out
for r in 1 2; do
  for v in new pf0; do
    lib=""; [ $v != new ] && lib=ab/$v.so
    BPE_LIB=$lib timeout -k 10 120 python3 tools/cp_time.py > $OUT/hpf_${v}_$r.log 2>&1 || exit 1
  done
done
echo done
