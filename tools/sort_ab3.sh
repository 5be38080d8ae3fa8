#!/usr/bin/env bash
# init sort passes: in-tree vs ab/sorthead.so vs timing diagnostics (ab/diag1:
# a plain coalesced copy in place of each chunk's sort; ab/diag2: the sort
# without its stores) -- init only, kernel times from rocprofv3
set -o pipefail
OUT=gpurun_out
export TMPDIR=/tmp BPE_GRAPH=0
for v in new head sortT512 sortT256 diag1 diag2; do
  lib=""; [ $v != new ] && lib=ab/$v.so; [ $v = head ] && lib=ab/sorthead.so
  BPE_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/sd_$v -o p -- python3 tools/sort_diag.py > $OUT/sd_$v.log 2>&1 || exit 1
done
echo done
