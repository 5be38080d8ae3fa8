#!/usr/bin/env bash
# round 4 checkpoint: the whole GPU suite, then the default bench line
set -o pipefail
OUT=gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/r4_gpu_tests_4.log 2>&1
echo "tests rc=$?" >> $OUT/r4_gpu_tests_4.log
grep -q "tests rc=0" $OUT/r4_gpu_tests_4.log || exit 1
timeout -k 10 800 python3 bench.py > $OUT/r4_bench_3.json 2> $OUT/r4_bench_3.err || exit 1
echo done
