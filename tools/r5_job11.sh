#!/usr/bin/env bash
# round 5: skip back-off + byte-pair-only relist staleness -- english-like
# variants, then configs[2] (bench, no extras) for batches / time / md5
set -o pipefail
OUT=gpurun_out
timeout -k 10 300 python -u tools/english_cmp.py 16 2000 > $OUT/r5_ecmp3.txt 2>&1 || { echo "cmp failed"; exit 1; }
timeout -k 10 200 python -u tools/english_dbg.py 16 1024 4096 > $OUT/r5_english8.txt 2>&1 || { echo "english dbg failed"; exit 1; }
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-encode > $OUT/r5_bench_a.json 2> $OUT/r5_bench_a.err || { echo "bench failed"; exit 1; }
echo done
