#!/usr/bin/env bash
# round 5: the creation-guess tie bound (BPE_TIE_UP=1) -- batches of
# configs[2] and train_1024
set -o pipefail
OUT=gpurun_out
BPE_TIE_UP=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-encode > $OUT/r5_bench_tieup.json 2> $OUT/r5_bench_tieup.err || { echo "bench tieup failed"; exit 1; }
echo done
