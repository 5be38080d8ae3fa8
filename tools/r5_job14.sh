#!/usr/bin/env bash
# round 5: the driver's default bench line on the current tree, then the
# second list (BPE_LIST2=1) on top of skipped keys
set -o pipefail
OUT=gpurun_out
timeout -k 10 600 python -u bench.py > $OUT/r5_bench_full.json 2> $OUT/r5_bench_full.err || { echo "bench failed"; exit 1; }
BPE_LIST2=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-encode > $OUT/r5_bench_list2.json 2> $OUT/r5_bench_list2.err || { echo "bench list2 failed"; exit 1; }
echo done
