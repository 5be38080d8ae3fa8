#!/usr/bin/env bash
# relist through the two-pass counting sort (default) vs the single-pass scatter
# (BPE_RELIST_SCATTER=1): configs[2] md5 / checksum / loop, kernel times, tests
set -o pipefail
OUT=gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for sc in 0 1; do
    BPE_RELIST_SCATTER=$sc timeout -k 10 120 python3 tools/batch_check.py 8192 > $OUT/rl_${sc}_$r.json 2>&1 || exit 1
  done
done
BPE_GRAPH=0 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/rlp -o p -- python3 tools/batch_check.py 8192 > $OUT/rlp.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py -x -q -k "rebuilds or config2" --timeout 300 --timeout-method thread > $OUT/rl_tests.log 2>&1 || exit 1
echo done
