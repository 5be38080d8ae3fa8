#!/usr/bin/env bash
# sort pass A at 8 waves per SIMD (two blocks per CU, 8 VGPRs spilled) vs the default
set -o pipefail
OUT=gpurun_out
export TMPDIR=/tmp BPE_GRAPH=0
for v in new sa8; do
  lib=""; [ $v != new ] && lib=ab/$v.so
  BPE_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/sd4_$v -o p -- python3 tools/sort_diag.py > $OUT/sd4_$v.log 2>&1 || exit 1
  BPE_LIB=$lib timeout -k 10 120 python3 tools/batch_check.py 1024 > $OUT/sd4_${v}_check.json 2>&1 || exit 1
done
echo done
