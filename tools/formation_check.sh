#!/usr/bin/env bash
# round 5: lane-parallel formation (tie check, membership) -- timelines,
# configs[2] batches / md5, batch tests
set -o pipefail
OUT=gpurun_out
BPE_DEBUG_TS=1 timeout -k 10 300 python -u bench.py --sharded --size 134217728 --merges 1024 --steps 2 --warmup 1 --no-cpu-baseline --no-encode --no-extras > $OUT/r5_ts_128c.txt 2>&1 || { echo "ts 128 failed"; exit 1; }
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-encode > $OUT/r5_bench_c.json 2> $OUT/r5_bench_c.err || { echo "bench failed"; exit 1; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_batch.py tests/test_gpu_parity.py > $OUT/r5_job17_tests.log 2>&1 || { echo "tests failed"; exit 1; }
echo done
