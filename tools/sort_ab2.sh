#!/usr/bin/env bash
# init sort passes: in-tree library vs ab/sorthead.so (init_ms + identical
# merges/ids, two rounds), kernel times of both, SQ counters of the in-tree one
set -o pipefail
OUT=gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for v in new head; do
    lib=""; [ $v = head ] && lib=ab/sorthead.so
    BPE_LIB=$lib timeout -k 10 120 python3 tools/batch_check.py 1024 > $OUT/sab_${v}_$r.json 2>&1 || exit 1
  done
done
for v in new head; do
  lib=""; [ $v = head ] && lib=ab/sorthead.so
  BPE_LIB=$lib BPE_GRAPH=0 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/sabp_$v -o p -- python3 tools/batch_check.py 16 > $OUT/sabp_$v.log 2>&1 || exit 1
done
tools/sort_pmc.sh || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $OUT/sab_parity.log 2>&1 || exit 1
echo done
