#!/usr/bin/env bash
# round 4: the three-shard divergence traced (BPE_DEBUG_FORM from merge 4440),
# then the count-sort rank step: LDS atomics (in-tree) vs wave multisplit
# (ab/sortms.so), kernel times from rocprofv3.
set -o pipefail
OUT=gpurun_out
export TMPDIR=/tmp
BPE_DEBUG_FORM=4440 timeout -k 10 200 python3 -u tools/shard3_dbg.py 4464 4465 1 > $OUT/shard3_trace.log 2>&1 || exit 1
for v in head sortms; do
  lib=""
  [ $v = sortms ] && lib=ab/sortms.so
  BPE_LIB=$lib timeout -k 10 120 python3 tools/batch_check.py 16 > $OUT/sort_$v.json 2>&1 || exit 1
  BPE_LIB=$lib timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/sortp_$v -o p -- python3 tools/batch_check.py 16 > $OUT/sortp_$v.log 2>&1 || exit 1
done
echo done
