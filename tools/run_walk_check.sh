#!/usr/bin/env bash
# the wave walk of long a == a runs: one-byte timing, then the run-heavy
# parity tests (single engine, batches, shards)
set -o pipefail
OUT=gpurun_out
timeout -k 10 200 python -u tools/onebyte_time.py > $OUT/onebyte2.log 2>&1 || { echo "timing failed"; exit 1; }
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_batch.py tests/test_gpu_shard.py > $OUT/run_walk_tests.log 2>&1 || { echo "tests failed"; exit 1; }
echo done
