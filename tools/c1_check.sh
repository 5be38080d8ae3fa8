#!/usr/bin/env bash
# configs[1]: per-merge timeline, then the one-merge engine's GPU tests
set -o pipefail
OUT=gpurun_out
BPE_DEBUG_TS=1 timeout -k 10 200 python3 tools/c1_prof.py > $OUT/c1_ts.json 2> $OUT/c1_ts.err || { echo "c1 ts failed"; exit 1; }
timeout -k 10 200 python3 tools/c1_prof.py > $OUT/c1_time.json 2> $OUT/c1_time.err || { echo "c1 time failed"; exit 1; }
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_spec.py tests/test_gpu_track.py tests/test_gpu_hot.py tests/test_gpu_parity.py > $OUT/c1_tests.log 2>&1 || { echo "tests failed"; exit 1; }
echo done
