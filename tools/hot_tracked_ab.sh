#!/usr/bin/env bash
# the hot set in tracked iterations (BPE_HOT_TRACKED=1, default) vs the level
# summaries (0): configs[1] time, the per-merge timeline, then the tracked /
# parity / hot tests
set -o pipefail
OUT=gpurun_out
for ht in 1 0; do
  BPE_HOT_TRACKED=$ht timeout -k 10 120 python3 tools/c1_prof.py > $OUT/ht_${ht}_1.json 2>&1 || exit 1
done
BPE_DEBUG_TS=1 timeout -k 10 120 python3 tools/c1_prof.py > $OUT/ht_ts.json 2> $OUT/ht_ts.err || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_track.py tests/test_gpu_parity.py tests/test_gpu_hot.py tests/test_gpu_mlog.py -x -q --timeout 250 --timeout-method thread > $OUT/ht_tests.log 2>&1 || exit 1
echo done
