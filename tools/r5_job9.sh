#!/usr/bin/env bash
# round 5: the english-like fixes (retry across stops, hot-set stride) --
# regression tests, variant comparison, then the corpus end to end and the
# batch / shard GPU tests
set -o pipefail
OUT=gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread \
  tests/test_gpu_batch.py -k "english_like or hot_set" > $OUT/r5_job9_english_tests.log 2>&1 || { echo "english tests failed"; exit 1; }
timeout -k 10 300 python -u tools/english_cmp.py 16 2000 > $OUT/r5_ecmp2.txt 2>&1 || { echo "cmp failed"; exit 1; }
timeout -k 10 200 python -u tools/english_dbg.py 16 64 1024 4096 > $OUT/r5_english5.txt 2>&1 || { echo "english dbg failed"; exit 1; }
timeout -k 10 300 python -u tools/init_skew.py 16 > $OUT/r5_init_skew.jsonl 2>&1 || { echo "init skew failed"; exit 1; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_batch.py tests/test_gpu_shard.py > $OUT/r5_job9_tests.log 2>&1 || { echo "batch/shard tests failed"; exit 1; }
echo done
